"""Cost of pinning a caller's pageable buffer in place (hipHostRegister / hipHostUnregister) against
copying it into pinned staging, and H2D bandwidth from each: is zero-copy DMA from the caller's
memory worth it at the host-buffer boundary? usage: python profiles/hostreg_probe.py [MiB=32] [reps=5]"""
import ctypes
import sys
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipDeviceSynchronize.argtypes = []


def ms(t0):
    return 1e3 * (time.perf_counter() - t0)


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = mib << 20
    d = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(d), n) == 0
    pinned = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(pinned), n, 0) == 0
    for r in range(reps):
        a = np.random.default_rng(r).integers(0, 255, n, dtype=np.uint8)  # fresh pageable, touched
        p = a.ctypes.data
        t0 = time.perf_counter()
        rc = hip.hipHostRegister(ctypes.c_void_p(p), n, 0)
        t_reg = ms(t0)
        t0 = time.perf_counter()
        hip.hipMemcpy(d, ctypes.c_void_p(p), n, 1)
        t_h2d_reg = ms(t0)
        t0 = time.perf_counter()
        hip.hipHostUnregister(ctypes.c_void_p(p))
        t_unreg = ms(t0)
        t0 = time.perf_counter()
        ctypes.memmove(pinned, p, n)
        t_copy = ms(t0)
        t0 = time.perf_counter()
        hip.hipMemcpy(d, pinned, n, 1)
        t_h2d_pin = ms(t0)
        t0 = time.perf_counter()
        hip.hipMemcpy(d, ctypes.c_void_p(p), n, 1)
        t_h2d_pageable = ms(t0)
        print(f"{mib} MiB: register rc={rc} {t_reg:.3f} ms, H2D from registered {t_h2d_reg:.3f} ms, unregister "
              f"{t_unreg:.3f} ms | memcpy to pinned (1 thread) {t_copy:.3f} ms, H2D from pinned {t_h2d_pin:.3f} ms | "
              f"H2D from pageable {t_h2d_pageable:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
