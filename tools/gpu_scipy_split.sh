cd "${GRAFT_REPO_ROOT}" && for c in c1 c2 c3; do for p in 0 1; do timeout -k 10 120 python tools/scipy_host_split.py --config $c --pipeline $p 2>&1 | grep -v amdgpu.ids || exit 1; done; done
