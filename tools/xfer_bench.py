"""Host <-> device transfer costs for the drop-in's end-to-end path (dev tool).

Times, for a 1 GiB f64 plane (512^3 x 8 B): D2H into fresh pageable memory (what
interpolate_field pays today), into pre-touched pageable memory, into hipHostMalloc'd memory
(and that allocation), and into hipHostRegister'ed numpy memory (and the registration).
usage: xfer_bench.py [GiB]
"""
import ctypes as C
import sys
import time

import numpy as np
import torch

GB = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
n = int(GB * (1 << 30))
hip = C.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostFree.argtypes = [C.c_void_p]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
hip.hipDeviceSynchronize.argtypes = []
D2H, H2D = 2, 1

dev = torch.empty(n // 8, dtype=torch.float64, device="cuda").fill_(1.0)
torch.cuda.synchronize()


def t(f):
    a = time.perf_counter()
    r = f()
    return (time.perf_counter() - a) * 1e3, r


def d2h(ptr):
    rc = hip.hipMemcpy(C.c_void_p(ptr), C.c_void_p(dev.data_ptr()), n, D2H)
    assert rc == 0, rc


out = {}
for rep in range(2):
    a = np.empty(n // 8)
    out[f"fresh_pageable_d2h_ms_{rep}"] = t(lambda: d2h(a.ctypes.data))[0]
    out[f"touched_pageable_d2h_ms_{rep}"] = t(lambda: d2h(a.ctypes.data))[0]
    del a
    p = C.c_void_p()
    out[f"hostmalloc_ms_{rep}"] = t(lambda: hip.hipHostMalloc(C.byref(p), n, 0))[0]
    out[f"pinned_d2h_ms_{rep}"] = t(lambda: d2h(p.value))[0]
    out[f"pinned_d2h2_ms_{rep}"] = t(lambda: d2h(p.value))[0]
    out[f"pinned_h2d_ms_{rep}"] = t(lambda: hip.hipMemcpy(C.c_void_p(dev.data_ptr()), p, n, H2D))[0]
    out[f"hostfree_ms_{rep}"] = t(lambda: hip.hipHostFree(p))[0]
    b = np.empty(n // 8)
    out[f"register_fresh_ms_{rep}"] = t(lambda: hip.hipHostRegister(C.c_void_p(b.ctypes.data), n, 0))[0]
    out[f"registered_d2h_ms_{rep}"] = t(lambda: d2h(b.ctypes.data))[0]
    out[f"unregister_ms_{rep}"] = t(lambda: hip.hipHostUnregister(C.c_void_p(b.ctypes.data)))[0]
    del b
    c = np.ones(n // 8)
    out[f"touch_then_register_ms_{rep}"] = t(lambda: hip.hipHostRegister(C.c_void_p(c.ctypes.data), n, 0))[0]
    hip.hipHostUnregister(C.c_void_p(c.ctypes.data))
    out[f"np_empty_touch_ms_{rep}"] = t(lambda: np.ones(n // 8))[0]
for kk, v in out.items():
    print(f"{kk:36s} {v:9.1f} ms  ({GB / (v * 1e-3):6.1f} GiB/s)")
