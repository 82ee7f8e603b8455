"""NTT-only timing (kgs_bench_ntt: forward + inverse pairs on a device buffer) of one library build,
selected with KGS_LIB: python profiles/ntt_ab.py LOGM REPS"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

import torch  # noqa: E402

K = importlib.import_module("kzg-grandsums-study_amd")


def main():
    logm, reps = int(sys.argv[1]), int(sys.argv[2])
    ctx = K.Context(0)
    g = torch.Generator().manual_seed(1)
    # canonical Montgomery-form elements: random 253-bit values (< r)
    x = torch.randint(0, 2**31 - 1, (1 << logm, 8), generator=g, dtype=torch.int64)
    x[:, 7] &= 0x0FFFFFFF
    d = x.to(torch.int32).cuda()
    ms = ctypes.c_double()
    L = K.lib()
    for _ in range(2):
        rc = L.kgs_bench_ntt(ctx._h, ctypes.c_void_p(d.data_ptr()), logm, reps, ctypes.byref(ms))
        assert rc == 0, K.lib().kgs_last_error()
    print(f"{os.environ.get('KGS_LIB', 'in-tree')}: 2^{logm} fwd+inv pair {ms.value / reps:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
