cd "$GRAFT_REPO_ROOT" || exit 1
for t in 6 10 14 16; do DHCOS_GEN_THREADS=$t timeout -k 10 120 python tools/gen_profile.py --reps 5 > /tmp/g.json 2>/dev/null || exit 1; python3 -c "
import json; d=json.load(open('/tmp/g.json')); print('threads $t', {k: round(d[k]*1e3,1) for k in ('draw','price','assemble','total','generate_synthetic_calibrations')})"; done
