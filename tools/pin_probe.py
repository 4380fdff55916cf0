"""Host-memory primitives for the generator's 1M-sample transfers: pinning a fresh 120 MB NumPy
array (hipHostRegister), a fresh pinned allocation (hipHostMalloc through libamdhip64), and copy
rates from pageable vs pinned memory."""
import ctypes as C
import time

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostFree.argtypes = [C.c_void_p]
torch.zeros(1, device="cuda")
NB = 120 * 2**20
for rep in range(3):
    a = np.empty(NB // 8)
    t0 = time.perf_counter()
    a.fill(0.0)
    t1 = time.perf_counter()
    rc = hip.hipHostRegister(a.ctypes.data, NB, 0)
    t2 = time.perf_counter()
    hip.hipHostUnregister(a.ctypes.data)
    t3 = time.perf_counter()
    b = np.empty(NB // 8)
    t4 = time.perf_counter()
    rc2 = hip.hipHostRegister(b.ctypes.data, NB, 0)
    t5 = time.perf_counter()
    hip.hipHostUnregister(b.ctypes.data)
    p = C.c_void_p()
    t6 = time.perf_counter()
    rc3 = hip.hipHostMalloc(C.byref(p), NB, 0)
    t7 = time.perf_counter()
    hip.hipHostFree(p)
    t8 = time.perf_counter()
    print(f"touch 120MB {1e3*(t1-t0):.2f} ms; register touched {1e3*(t2-t1):.2f} (rc {rc}), unregister "
          f"{1e3*(t3-t2):.2f}; register untouched {1e3*(t5-t4):.2f} (rc {rc2}); hipHostMalloc "
          f"{1e3*(t7-t6):.2f} (rc {rc3}), free {1e3*(t8-t7):.2f}")
