#!/bin/bash
# Host-side generator timings on this host (run on the GPU box via gpurun): the native draw's
# passes ($DHCOS_GEN_TIMING) and the native assembly at several worker counts
# ($DHCOS_GEN_THREADS), 1M samples x 15 options as tools/gen_profile.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for t in ${THREADS:-1 4 16}; do
  DHCOS_GEN_THREADS=$t DHCOS_GEN_TIMING=1 timeout -k 10 120 python3 -c "
import sys, time, numpy as np
sys.path.insert(0, 'option-pricing-ffn-lbfgs_amd')
from dhcos import generator as G, _native
for r in range(3):
    np.random.seed(0)
    t0 = time.perf_counter(); p, s, nz = G.draw_paths(1000000); t1 = time.perf_counter()
    _native.gen_assemble(np.abs(nz) + 1.0, nz, s, np.linspace(80.0, 120.0, nz.shape[1]))
    t2 = time.perf_counter()
    print('threads $t: draw_paths %.4f s, gen_assemble %.4f s' % (t1 - t0, t2 - t1))
" || exit 1
done
