"""kzg-grandsums-study_amd — MI355X-native KZG grand-sum / grand-product prover (host mirror).

Python mirror of the reference's module API (xavi-pinsach/kzg-grandsums-study):

    prover(pTauFilename, evalsFs, evalsTs, evalsSelF=None, evalsSelT=None) -> proof
        src/grandsum/mset_eq_kzg_prover.js:12  -> grandsum_prover
        src/grandproduct/mset_eq_kzg_prover.js:12 -> grandproduct_prover
    lookup_prover(pTauFilename, evalsFs, evalsTs, evalsSelF, evalsMulT) -> proof
        test/lookup_kzg_grandsum.test.js:24-44 (commented out in the reference) -> KGS_LOOKUP

over the C-ABI library lib/libkgs.so (include/kgs.h; HIP kernels for gfx950). The JavaScript
drop-in modules (js/) bind the same library through an N-API addon. There is NO CPU fallback:
if the HIP library cannot be loaded the import raises.

Input/ownership conventions follow the reference exactly: F/T evaluations are
32 B LE standard-form buffers that are overwritten with their Montgomery form (prover.js:147-148);
selectors are Montgomery buffers; the proof is {"commitments": {name: 64 B LEM},
"evaluations": {name: 32 B LE Montgomery}}.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KGS_LIB") or os.path.join(_HERE, "lib", "libkgs.so")

GRANDSUM = 0
GRANDPRODUCT = 1
LOOKUP = 2

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
FR_ONE_MONT = ((1 << 256) % R).to_bytes(32, "little")

_lib = None


class KgsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


KGS_E_RANGE = -9


class RangeError(ValueError):
    """What the reference's JavaScript throws as a RangeError ("offset is out of bounds": its divZh on a
    zero quotient, polynomial.js:857,884) — raised in reference-quirks mode only (include/kgs.h
    kgs_ctx_set_reference_quirks)."""


def _semantic(e):
    """KgsError from the library -> the exception the reference's prover would throw."""
    return RangeError(str(e)) if e.code == KGS_E_RANGE else ValueError(str(e))


def lib():
    """Load lib/libkgs.so (raises if it is missing: the HIP path is the only path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        c_u8p = ctypes.c_void_p
        L.kgs_last_error.restype = ctypes.c_char_p
        L.kgs_version.restype = ctypes.c_char_p
        L.kgs_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.kgs_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.kgs_ctx_destroy.restype = None
        L.kgs_srs_load_ptau.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.kgs_srs_load_ptau_slice.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.kgs_srs_slice_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_uint64)]
        L.kgs_ptau_power.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        L.kgs_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.kgs_srs_load_points.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.kgs_srs_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_int)]
        L.kgs_ptau_read_tau_g2.argtypes = [ctypes.c_char_p, c_u8p]
        L.kgs_ptau_write_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, c_u8p]
        PP = ctypes.POINTER(ctypes.c_void_p)
        L.kgs_prove.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, PP, PP, c_u8p, c_u8p,
                                PP, PP, c_u8p, c_u8p]
        L.kgs_prove_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, PP, PP,
                                       ctypes.c_void_p, ctypes.c_void_p, c_u8p, c_u8p]
        L.kgs_proof_shape.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_int)]
        L.kgs_host_register.argtypes = [c_u8p, ctypes.c_uint64]
        L.kgs_host_unregister.argtypes = [c_u8p]
        L.kgs_last_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.kgs_ctx_idle.argtypes = [ctypes.c_void_p]
        L.kgs_fr_to_mont.argtypes = [ctypes.c_void_p, c_u8p, c_u8p, ctypes.c_uint64]
        L.kgs_fr_from_mont.argtypes = [ctypes.c_void_p, c_u8p, c_u8p, ctypes.c_uint64]
        L.kgs_fr_batch_inverse.argtypes = [ctypes.c_void_p, c_u8p, c_u8p, ctypes.c_uint64]
        L.kgs_ntt.argtypes = [ctypes.c_void_p, c_u8p, c_u8p, ctypes.c_int, ctypes.c_int]
        L.kgs_msm.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, c_u8p]
        L.kgs_grand_build.argtypes = [ctypes.c_void_p, ctypes.c_int, c_u8p, c_u8p, c_u8p, c_u8p, c_u8p,
                                      ctypes.c_uint64, c_u8p]
        L.kgs_poly_eval.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, c_u8p, c_u8p]
        L.kgs_poly_div_x_sub.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, c_u8p, c_u8p]
        L.kgs_keccak256.argtypes = [c_u8p, ctypes.c_uint64, c_u8p]
        L.kgs_bench_msm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double)]
        L.kgs_bench_msm_phases.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
        L.kgs_bench_ntt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double)]
        L.kgs_verify.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_u8p, c_u8p, c_u8p]
        L.kgs_verify_ptau.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_u8p,
                                      c_u8p]
        L.kgs_ctx_set_shard.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.kgs_ctx_set_msm_lanes.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.kgs_ctx_set_reference_quirks.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.kgs_shard_range.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]
        L.kgs_msm_combine.argtypes = [c_u8p, ctypes.c_int, ctypes.c_int, c_u8p]
        L.kgs_group_create_local.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.kgs_group_create_host.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_void_p)]
        L.kgs_group_create_host_a2a.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.POINTER(ctypes.c_void_p)]
        L.kgs_last_exchange.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.kgs_group_rccl_unique_id.argtypes = [c_u8p]
        L.kgs_group_create_rccl.argtypes = [ctypes.c_int, ctypes.c_int, c_u8p, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_void_p)]
        L.kgs_group_destroy.argtypes = [ctypes.c_void_p]
        L.kgs_group_destroy.restype = None
        L.kgs_group_world.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.kgs_ctx_set_group.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


# int (*kgs_allgather_fn)(void* user, const uint8_t* send, uint8_t* recv, uint64_t bytes)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
# int (*kgs_alltoall_fn)(void* user, const uint8_t* send, uint8_t* recv, uint64_t chunk)
ALLTOALL_FN = ALLGATHER_FN


def _check(rc):
    if rc < 0:
        raise KgsError(rc, lib().kgs_last_error().decode())
    return rc


def _buf(b):
    """bytes-like -> (ctypes buffer, pointer) keeping it alive."""
    cb = ctypes.create_string_buffer(bytes(b), len(b)) if b is not None else None
    return cb


_PBA = ctypes.pythonapi.PyByteArray_FromStringAndSize
_PBA.restype = ctypes.py_object
_PBA.argtypes = [ctypes.c_char_p, ctypes.c_ssize_t]


def _uninit_bytearray(n):
    """bytearray of n bytes WITHOUT the zero fill of bytearray(n) (CPython C API; the library
    overwrites every byte): saves a 32 MiB memset per written-back vector at n = 2^20."""
    return _PBA(None, n)


def _ptr(b):
    """Zero-copy pointer to a bytes-like object's memory: (pointer, keep-alive). bytes are read
    in place (c_char_p); writable buffers (bytearray, numpy) through from_buffer; anything else
    is copied once."""
    if isinstance(b, bytes):
        cp = ctypes.c_char_p(b)
        return ctypes.cast(cp, ctypes.c_void_p), (b, cp)
    try:
        arr = (ctypes.c_char * len(b)).from_buffer(b)
        return ctypes.cast(arr, ctypes.c_void_p), (b, arr)
    except (TypeError, ValueError):
        cb = ctypes.create_string_buffer(bytes(b), len(b))
        return ctypes.cast(cb, ctypes.c_void_p), cb


def keccak256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    src = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    _check(lib().kgs_keccak256(src, len(data), out))
    return out.raw


def ptau_power(path):
    """Power of a ptau file, from its header only (kgs_ptau_power; readPTauHeader, ptau_utils.js:3-24)."""
    p = ctypes.c_int()
    _check(lib().kgs_ptau_power(os.fsencode(path), ctypes.byref(p)))
    return p.value


def device_count():
    n = ctypes.c_int()
    _check(lib().kgs_device_count(ctypes.byref(n)))
    return n.value


def host_register(buf):
    """Pin a writable host buffer (bytearray / numpy) that several proofs will reuse: kgs_prove then
    DMAs it in place instead of through pinned staging (kgs_host_register). Returns a handle to pass
    to host_unregister before the buffer is released or resized."""
    p, keep = _ptr(buf)
    if isinstance(keep, ctypes.Array):
        raise TypeError("host_register needs a writable buffer (bytearray, numpy array)")
    _check(lib().kgs_host_register(p, len(buf)))
    return p, keep


def host_unregister(handle):
    _check(lib().kgs_host_unregister(handle[0]))


def shard_range(n, rank, world):
    """Point range [lo, hi) of an n-point MSM owned by `rank` (kgs_shard_range)."""
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().kgs_shard_range(n, rank, world, ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def msm_combine(T_all, nparts, c):
    """Commitment (64 B affine LEM) from `nparts` rank partials of c XYZZ bit-sum points each."""
    if len(T_all) != nparts * c * 128:
        raise ValueError("T_all must hold nparts * c * 128 bytes")
    out = ctypes.create_string_buffer(64)
    _check(lib().kgs_msm_combine(_buf(T_all), nparts, c, out))
    return out.raw


def torch_allgather(group=None, device=None):
    """All-gather transport for Context.set_shard over torch.distributed: RCCL (backend "nccl")
    when `device` is a GPU, gloo on host tensors otherwise."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)

    def fn(data):
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        if device is not None:
            t = t.to(device)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        return b"".join(o.cpu().numpy().tobytes() for o in outs)
    return fn


def torch_alltoall(group=None):
    """All-to-all transport for Group.host over torch.distributed (all_to_all_single on host tensors:
    gloo): alltoall(data, chunk) sends chunk j of `data` to rank j and returns the world chunks
    received, rank-major."""
    import torch
    import torch.distributed as dist

    def fn(data, chunk):
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t, group=group)
        return out.numpy().tobytes()
    return fn


class Group:
    """Rank group of the distributed prover (kgs_group_t; Context.set_group): every vector of a
    proof sharded over `world` ranks, one context per rank.
      Group.local(world)                 several contexts of this process (one host thread per rank)
      Group.host(world, allgather[, alltoall])
                                         any host all-gather(bytes) -> world * bytes (e.g. gloo) and,
                                         optionally, an all-to-all(bytes, chunk) -> bytes (chunk j to
                                         rank j: (W - 1) / W of a vector leaves a rank instead of every
                                         rank receiving W x it); device data is staged through the host
      Group.rccl(rank, world, id, dev)   one process per GPU, RCCL over xGMI; id = rccl_unique_id()
                                         made on rank 0 and broadcast by the caller"""

    def __init__(self, handle, world, keep=None):
        self._h = handle
        self.world = world
        self._keep = keep

    @classmethod
    def local(cls, world):
        h = ctypes.c_void_p()
        _check(lib().kgs_group_create_local(world, ctypes.byref(h)))
        return cls(h, world)

    @classmethod
    def host(cls, world, allgather, alltoall=None):
        def _cb(user, send, recv, nbytes):
            try:
                out = allgather(ctypes.string_at(send, nbytes))
                if len(out) != nbytes * world:
                    return -1
                ctypes.memmove(recv, out, len(out))
                return 0
            except Exception:  # reported to the caller as KGS_E_COMM
                import traceback
                traceback.print_exc()
                return -1

        def _a2a(user, send, recv, chunk):
            try:
                out = alltoall(ctypes.string_at(send, chunk * world), chunk)
                if len(out) != chunk * world:
                    return -1
                ctypes.memmove(recv, out, len(out))
                return 0
            except Exception:
                import traceback
                traceback.print_exc()
                return -1
        cb = ALLGATHER_FN(_cb)
        h = ctypes.c_void_p()
        if alltoall is None:
            _check(lib().kgs_group_create_host(world, ctypes.cast(cb, ctypes.c_void_p), None, ctypes.byref(h)))
            return cls(h, world, cb)
        cb2 = ALLTOALL_FN(_a2a)
        _check(lib().kgs_group_create_host_a2a(world, ctypes.cast(cb, ctypes.c_void_p), ctypes.cast(cb2, ctypes.c_void_p),
                                               None, ctypes.byref(h)))
        return cls(h, world, (cb, cb2))

    @classmethod
    def rccl(cls, rank, world, uid, device):
        h = ctypes.c_void_p()
        _check(lib().kgs_group_create_rccl(rank, world, _buf(uid), device, ctypes.byref(h)))
        return cls(h, world)

    def close(self):
        if self._h:
            lib().kgs_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rccl_unique_id():
    """128-byte RCCL communicator id (kgs_group_rccl_unique_id), made on rank 0 and broadcast."""
    out = ctypes.create_string_buffer(128)
    _check(lib().kgs_group_rccl_unique_id(out))
    return out.raw


class ThreadGroup:
    """In-process all-gather between `world` contexts driven by `world` host threads (one rank
    each): several GPUs of one process, or the sharded path rehearsed on a single GPU."""

    def __init__(self, world):
        import threading
        self.world = world
        self._bar = threading.Barrier(world)
        self._slots = [None] * world

    def allgather(self, rank):
        def fn(data):
            self._slots[rank] = bytes(data)
            self._bar.wait()
            out = b"".join(self._slots)
            self._bar.wait()
            return out
        return fn


class Evaluations:
    """Mirror of src/polynomial/evaluations.js (the prover's input container): `.eval` bytes."""

    def __init__(self, eval_bytes):
        self.eval = bytes(eval_bytes)

    def length(self):
        if len(self.eval) % 32:
            raise ValueError("Polynomial evaluations buffer has incorrect size")
        return len(self.eval) // 32

    @staticmethod
    def getOneEvals(length):
        return Evaluations(FR_ONE_MONT * length)

    def isAllOnes(self):
        return self.eval == FR_ONE_MONT * self.length()

    def isAllZeros(self):
        return self.eval == bytes(len(self.eval))


class Context:
    """One HIP device + resident SRS. Not re-entrant (like the reference's curve object)."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        _check(lib().kgs_ctx_create(device, ctypes.byref(self._h)))
        self._srs = None

    def close(self):
        if self._h:
            lib().kgs_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_reference_quirks(self, on):
        """Reference-quirks mode (kgs_ctx_set_reference_quirks; default ON unless the environment has
        KGS_REFERENCE_QUIRKS == "0"): reproduce the reference's failures on degenerate inputs; off, the
        exact-math prover proves them."""
        _check(lib().kgs_ctx_set_reference_quirks(self._h, 1 if on else 0))

    def set_msm_lanes(self, lanes):
        """1 or 2 HIP streams for the independent MSMs of a prover round (kgs_ctx_set_msm_lanes)."""
        _check(lib().kgs_ctx_set_msm_lanes(self._h, lanes))

    def set_shard(self, rank, world, allgather=None):
        """MSM point-range sharding (kgs_ctx_set_shard): `allgather(bytes) -> world * bytes`
        (rank-major), called in the same order on every rank. world == 1 switches it off."""
        if world > 1 and allgather is None:
            raise ValueError("sharding needs an all-gather transport")

        def _cb(user, send, recv, nbytes):
            try:
                out = allgather(ctypes.string_at(send, nbytes))
                if len(out) != nbytes * world:
                    return -1
                ctypes.memmove(recv, out, len(out))
                return 0
            except Exception:  # reported to the caller as KGS_E_COMM
                import traceback
                traceback.print_exc()
                return -1
        self._shard_cb = ALLGATHER_FN(_cb) if world > 1 else None
        fp = ctypes.cast(self._shard_cb, ctypes.c_void_p) if world > 1 else None
        _check(lib().kgs_ctx_set_shard(self._h, rank, world, fp, None))

    def set_group(self, group, rank=0):
        """Attach the distributed prover (kgs_ctx_set_group): this context is `rank` of `group`;
        None detaches. Keeps the group alive while attached."""
        _check(lib().kgs_ctx_set_group(self._h, group._h if group is not None else None, rank))
        self._group = group

    def load_ptau(self, path, nbits_max=-1, slice=None):
        """kgs_srs_load_ptau; slice=(rank, world): only rank's slice of the SRS, the points rank + world*j
        (kgs_srs_load_ptau_slice) — what a rank of the distributed prover commits with"""
        if slice is None:
            _check(lib().kgs_srs_load_ptau(self._h, os.fsencode(path), nbits_max))
        else:
            _check(lib().kgs_srs_load_ptau_slice(self._h, os.fsencode(path), nbits_max, int(slice[0]), int(slice[1])))
        self._srs = (path, nbits_max, slice)

    def srs_slice_info(self):
        """(rank, world, window-table bytes) of the resident SRS (world 1: the whole prefix)"""
        r, w, b = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint64()
        _check(lib().kgs_srs_slice_info(self._h, ctypes.byref(r), ctypes.byref(w), ctypes.byref(b)))
        return r.value, w.value, b.value

    def srs_info(self):
        p, c = ctypes.c_int(), ctypes.c_int()
        n = ctypes.c_uint64()
        _check(lib().kgs_srs_info(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(c)))
        return p.value, n.value, c.value

    def write_synthetic_ptau(self, path, power, tau):
        t = ctypes.create_string_buffer(int(tau % R).to_bytes(32, "little"), 32)
        _check(lib().kgs_ptau_write_synthetic(self._h, os.fsencode(path), power, t))

    # ---- primitives (host buffers) ----
    def fr_to_mont(self, data):
        n = len(data) // 32
        out = ctypes.create_string_buffer(32 * n)
        _check(lib().kgs_fr_to_mont(self._h, _buf(data), out, n))
        return out.raw

    def fr_from_mont(self, data):
        n = len(data) // 32
        out = ctypes.create_string_buffer(32 * n)
        _check(lib().kgs_fr_from_mont(self._h, _buf(data), out, n))
        return out.raw

    def fr_batch_inverse(self, data):
        n = len(data) // 32
        out = ctypes.create_string_buffer(32 * n)
        _check(lib().kgs_fr_batch_inverse(self._h, _buf(data), out, n))
        return out.raw

    def ntt(self, data, inverse=False):
        m = len(data) // 32
        logm = m.bit_length() - 1
        out = ctypes.create_string_buffer(32 * m)
        _check(lib().kgs_ntt(self._h, _buf(data), out, logm, 1 if inverse else 0))
        return out.raw

    def msm(self, scalars_mont):
        n = len(scalars_mont) // 32
        out = ctypes.create_string_buffer(64)
        _check(lib().kgs_msm(self._h, _buf(scalars_mont) if n else None, n, out))
        return out.raw

    def grand_build(self, kind, f_mont, t_mont, gamma_mont, sel_f=None, sel_t=None):
        n = len(f_mont) // 32
        out = ctypes.create_string_buffer(32 * n)
        _check(lib().kgs_grand_build(self._h, kind, _buf(f_mont), _buf(t_mont), _buf(sel_f), _buf(sel_t),
                                     _buf(gamma_mont), n, out))
        return out.raw

    def poly_eval(self, coef_mont, x_mont):
        out = ctypes.create_string_buffer(32)
        _check(lib().kgs_poly_eval(self._h, _buf(coef_mont), len(coef_mont) // 32, _buf(x_mont), out))
        return out.raw

    def poly_div_x_sub(self, coef_mont, z_mont):
        out = ctypes.create_string_buffer(len(coef_mont))
        _check(lib().kgs_poly_div_x_sub(self._h, _buf(coef_mont), len(coef_mont) // 32, _buf(z_mont), out))
        return out.raw

    def last_exchange(self):
        """Exchanges of the last proof (kgs_last_exchange): all-to-all count / summed span ms / bytes
        sent, host all-gather count / wall ms / bytes sent; zeros after a single-GPU proof."""
        arr = (ctypes.c_double * 6)()
        lib().kgs_last_exchange(self._h, arr, 6)
        return {"alltoall_n": int(arr[0]), "alltoall_ms": arr[1], "alltoall_bytes": int(arr[2]),
                "allgather_n": int(arr[3]), "allgather_ms": arr[4], "allgather_bytes": int(arr[5])}

    def idle(self):
        """True when none of the context's streams has work outstanding (kgs_ctx_idle)."""
        rc = lib().kgs_ctx_idle(self._h)
        _check(rc)
        return rc == 1

    def last_timing(self):
        arr = (ctypes.c_double * 9)()
        n = lib().kgs_last_timing(self._h, arr, 9)
        return list(arr[:max(n, 0)])

    # ---- full prover ----
    def prove(self, kind, nbits, evals_f, evals_t, sel_f=None, sel_t=None, mont_out=True):
        """Host-buffer prover; returns (commitment list, evaluation list, mont_f, mont_t). Inputs
        are read in place; the Montgomery forms come back as bytearrays (no extra copies).
        mont_out: True (new bytearrays), False (no write-back), or a pair of lists (mont_f, mont_t)
        of writable caller buffers of 32 * 2^nbits bytes each that receive the Montgomery forms (a
        caller that recycles its output buffers, as the JS module's pool does)."""
        k = len(evals_f)
        n = 1 << nbits
        if any(len(x) != 32 * n for x in list(evals_f) + list(evals_t)):
            raise ValueError("evaluation buffers must hold 2^nbits 32-byte elements")
        given = None
        if isinstance(mont_out, (tuple, list)):
            given = (list(mont_out[0]), list(mont_out[1]))
            if len(given[0]) != k or len(given[1]) != k or any(len(x) != 32 * n for x in given[0] + given[1]):
                raise ValueError("write-back buffers must be two lists of npols buffers of 2^nbits 32-byte elements")
        keep = []
        PF = (ctypes.c_void_p * k)()
        PT = (ctypes.c_void_p * k)()
        MF = (ctypes.c_void_p * k)()
        MT = (ctypes.c_void_p * k)()
        mf, mt = [], []
        for i in range(k):
            (pf, kf), (pt, kt) = _ptr(evals_f[i]), _ptr(evals_t[i])
            keep += [kf, kt]
            PF[i], PT[i] = pf, pt
            if mont_out:
                ma, mb = (given[0][i], given[1][i]) if given else (_uninit_bytearray(32 * n), _uninit_bytearray(32 * n))
                (pa, ka), (pb, kb) = _ptr(ma), _ptr(mb)
                keep += [ka, kb]
                mf.append(ma)
                mt.append(mb)
                MF[i], MT[i] = pa, pb
        selected = sel_f is not None
        nc, ne = ctypes.c_int(), ctypes.c_int()
        lib().kgs_proof_shape(kind, k, 1 if selected else 0, ctypes.byref(nc), ctypes.byref(ne))
        com = ctypes.create_string_buffer(64 * nc.value)
        ev = ctypes.create_string_buffer(32 * ne.value)
        sf = st = None
        if selected:
            (sf, ksf), (st, kst) = _ptr(sel_f), _ptr(sel_t)
            keep += [ksf, kst]
        _check(lib().kgs_prove(self._h, kind, nbits, k, PF, PT, sf, st, MF if mont_out else None,
                               MT if mont_out else None, com, ev))
        coms = [com.raw[64 * i:64 * i + 64] for i in range(nc.value)]
        evs = [ev.raw[32 * i:32 * i + 32] for i in range(ne.value)]
        return coms, evs, mf, mt

    def prove_device(self, kind, nbits, d_f, d_t, d_sf=None, d_st=None):
        """Device-resident prover (d_* are device pointers as ints). Returns (commitments, evaluations)."""
        k = len(d_f)
        PF = (ctypes.c_void_p * k)(*d_f)
        PT = (ctypes.c_void_p * k)(*d_t)
        selected = d_sf is not None
        nc, ne = ctypes.c_int(), ctypes.c_int()
        lib().kgs_proof_shape(kind, k, 1 if selected else 0, ctypes.byref(nc), ctypes.byref(ne))
        com = ctypes.create_string_buffer(64 * nc.value)
        ev = ctypes.create_string_buffer(32 * ne.value)
        _check(lib().kgs_prove_device(self._h, kind, nbits, k, PF, PT, d_sf, d_st, com, ev))
        return ([com.raw[64 * i:64 * i + 64] for i in range(nc.value)],
                [ev.raw[32 * i:32 * i + 32] for i in range(ne.value)])


def dist_exchange_model(kind, nbits, npols, selected, world):
    """All-to-alls of one distributed proof (csrc/prover_dist.cpp) and the bytes that
    leave each rank in them: round 1 one per F_i / T_i (+ selectors) at n; round 2 S BLOCK -> E and its
    inverse at n, the coset forward transforms of S, F, T (+ selectors) at the coset size cs; round 3
    the quotient's inverse at cs; round 5 the two numerators CYCLIC -> BLOCK and the two openings
    BLOCK -> CYCLIC (one at cs, one at n each). An all-to-all of a length-L vector sends L / W^2
    elements to each of the W - 1 other ranks."""
    n = 1 << nbits
    gs = kind != GRANDPRODUCT
    cs = n if (not gs and not selected) else 2 * n
    sel = 2 if selected else 0
    lens = [n] * (2 * npols + sel) + [n, n] + [cs] * (3 + sel) + [cs] + [cs, n, cs, n]
    W = world
    return {"alltoall_n": len(lens), "alltoall_bytes": sum(32 * (L // (W * W)) * (W - 1) for L in lens)}


def proof_names(kind, npols, selected):
    """Commitment / evaluation key order of the C-ABI outputs (kgs.h) in the reference's names."""
    vec = npols > 1
    gs = kind != GRANDPRODUCT
    com = []
    for i in range(npols):
        com += [f"F{i}" if vec else "F", f"T{i}" if vec else "T"]
    if selected:
        com += ["selF", "selT"]
    com += ["S" if gs else "Z", "Q", "Wxi", "Wxiw"]
    ev = []
    for i in range(npols):
        ev.append(f"f{i}xi" if vec else "fxi")
        if gs:
            ev.append(f"t{i}xi" if vec else "txi")
    if selected:
        ev += ["selFxi", "selTxi"]
    ev.append("sxiw" if gs else "zxiw")
    return com, ev


_CTX = {}


def _context(device=0):
    if device not in _CTX:
        _CTX[device] = Context(device)
    return _CTX[device]


def _prover(kind, pTauFilename, evalsFs, evalsTs, evalsSelF=None, evalsSelT=None, device=0):
    """src/grandsum/mset_eq_kzg_prover.js:12-142 — input checks with the reference's messages, then
    the HIP prover. Overwrites evalsFs[i].eval / evalsTs[i].eval with Montgomery form (:147-148)."""
    log.info("> MULTISET EQUALITY KZG %s PROVER STARTED", _TITLE[kind])
    power = ptau_power(pTauFilename)  # the header is read first (prover.js:15-16)
    if not isinstance(evalsFs, (list, tuple)):
        evalsFs = [evalsFs]
    if not isinstance(evalsTs, (list, tuple)):
        evalsTs = [evalsTs]
    if len(evalsFs) != len(evalsTs):
        raise ValueError("The lengths of the two vector multisets must be the same.")
    npols = len(evalsFs)
    if npols == 0:
        raise ValueError("The number of multisets must be greater than 0.")
    for i in range(npols):
        if evalsFs[i].length() != evalsTs[i].length():
            raise ValueError(f"The {i}-th multiset buffers must have the same length.")
        elif evalsFs[i].length() != evalsFs[0].length():
            raise ValueError("The multiset buffers must all have the same length.")
    n0 = evalsFs[0].length()
    if kind == LOOKUP and evalsSelT is None:
        raise ValueError("A lookup needs the multiplicities of the table.")
    if evalsSelF is None:
        evalsSelF = Evaluations.getOneEvals(n0)
    if evalsSelT is None:
        evalsSelT = Evaluations.getOneEvals(n0)
    if evalsSelF.length() != evalsSelT.length():
        raise ValueError("The selection buffers must have the same length.")
    elif evalsSelF.length() != n0:
        raise ValueError("The selection buffers must have the same length as the multiset buffers.")
    # a lookup keeps its selectors even when all one (its proof always carries selF / selT)
    is_selected = kind == LOOKUP or not (evalsSelF.isAllOnes() and evalsSelT.isAllOnes())
    if is_selected and evalsSelF.isAllZeros() and evalsSelT.isAllZeros():  # prover.js:66-68
        log.warning("The selection buffers are all zeros. The argument is trivially satisfied.")
    nbits = (n0 - 1).bit_length() if n0 > 0 else 0
    if n0 != (1 << nbits):
        raise ValueError("Polynomial length must be a power of two.")
    if power < nbits:
        raise ValueError("The Powers of Tau file is not sufficiently large to commit the polynomials.")
    if log.isEnabledFor(logging.INFO):  # prover.js:87-93
        for line in ("-------------------------------------", f"  MULTISET EQUALITY KZG {_TITLE[kind]} PROVER SETTINGS",
                     "  Curve:       bn128", f"  Domain size: {1 << nbits}", f"  Number of polynomials: {npols}",
                     f"  Selectors: {'Yes' if is_selected else 'No'}", "-------------------------------------"):
            log.info(line)
    ctx = _context(device)
    # the drop-in functions follow the environment on every call (contexts are cached per device)
    ctx.set_reference_quirks(os.environ.get("KGS_REFERENCE_QUIRKS", "1") != "0")
    # only the 2^(nbits+1) points this proof commits with (prover.js:83-85); grow-only device cache
    ctx.load_ptau(pTauFilename, nbits)
    coms, evs, mf, mt = ctx.prove(kind, nbits, [e.eval for e in evalsFs], [e.eval for e in evalsTs],
                                  evalsSelF.eval if is_selected else None,
                                  evalsSelT.eval if is_selected else None)
    for i in range(npols):
        evalsFs[i].eval = mf[i]
        evalsTs[i].eval = mt[i]
    cn, en = proof_names(kind, npols, is_selected)
    proof = {"commitments": dict(zip(cn, coms)), "evaluations": dict(zip(en, evs))}
    if log.isEnabledFor(logging.INFO):
        log_rounds(kind, proof, nbits, npols, is_selected)
    return proof


# ---------------------------------------------------------------- the reference's log lines
# logger.js (logplease at INFO) as used by src/grandsum/mset_eq_kzg_prover.js:13-140,164-412 and the
# grand-product twin: the same messages on the standard `logging` logger "kgs" (silent until the
# caller enables INFO on it). The proof is computed in one library call, so the round lines follow
# it, with the challenges replayed from the proof's transcript (src/Keccak256Transcript.js:7-53).
import logging  # noqa: E402

log = logging.getLogger("kgs")
_FQ = 21888242871839275222246405745257275088696311157297823662689037894645226208583
_FR = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_TITLE = {GRANDSUM: "GRAND-SUM", GRANDPRODUCT: "GRAND-PRODUCT", LOOKUP: "GRAND-SUM (LOOKUP)"}


def _fr_int(b):  # 32 B LE Montgomery Fr -> integer
    return int.from_bytes(bytes(b), "little") * pow(1 << 256, _FR - 2, _FR) % _FR


def _g1_xy(b):  # 64 B affine LEM -> (x, y) standard, None for the zero point
    rinv = pow(1 << 256, _FQ - 2, _FQ)
    x = int.from_bytes(bytes(b[:32]), "little") * rinv % _FQ
    y = int.from_bytes(bytes(b[32:64]), "little") * rinv % _FQ
    return None if x == 0 and y == 0 else (x, y)


def _g1_str(b):  # [ffjs] G1.toString of an affine point
    a = _g1_xy(b)
    return "[ 0, 1, 0 ]" if a is None else f"[ {a[0]}, {a[1]}, 1 ]"


class _Transcript:
    """G1.toRprUncompressed (64 B big-endian x||y, the zero point 0x40 then zeros) / Fr.toRprBE (32 B);
    a challenge is keccak256 of everything added so far, big-endian, mod r."""

    def __init__(self):
        self.buf = bytearray()

    def add_commitment(self, b):
        a = _g1_xy(b)
        self.buf += (b"\x40" + bytes(63)) if a is None else a[0].to_bytes(32, "big") + a[1].to_bytes(32, "big")

    def add_scalar(self, v):
        self.buf += (v % _FR).to_bytes(32, "big")

    def challenge(self):
        return int.from_bytes(keccak256(bytes(self.buf)), "big") % _FR


def log_rounds(kind, proof, nbits, npols, selected, logger=None):
    """Write the reference's round log of `proof` (prover.js:111-140 with each round's lines) and
    return its challenges {beta, gamma, alpha, xi, v} (beta None for k = 1)."""
    lg = logger or log
    gs = kind != GRANDPRODUCT
    vec = npols > 1
    C, E = proof["commitments"], proof["evaluations"]
    tr = _Transcript()
    msg = "> ROUND ${round}. Generate the witness polynomials"  # printed literally by the reference
    msg += f" fᵢ,tᵢ ∈ 𝔽[X], for i ∈ [{npols}]" if vec else " f,t ∈ 𝔽[X]"
    if selected:
        msg += ", and the selector polynomials fsel,tsel ∈ 𝔽[X]"
    lg.info(msg)
    for i in range(npols):
        nf, nt = (f"F{i}", f"T{i}") if vec else ("F", "T")
        lg.info("··· [%s]₁ = %s", f"f{i + 1}(x)" if vec else "f(x)", _g1_str(C[nf]))
        lg.info("··· [%s]₁ = %s", f"t{i + 1}(x)" if vec else "t(x)", _g1_str(C[nt]))
        tr.add_commitment(C[nf])
        tr.add_commitment(C[nt])
    if selected:
        lg.info("··· [fsel(x)]₁ = %s", _g1_str(C["selF"]))
        lg.info("··· [tsel(x)]₁ = %s", _g1_str(C["selT"]))
        tr.add_commitment(C["selF"])
        tr.add_commitment(C["selT"])
    sz = "S" if gs else "Z"
    lg.info("> ROUND 2. Compute the grand-%s polynomial %s ∈ 𝔽[X]", "sum" if gs else "product", sz)
    beta = None
    if vec:
        beta = tr.challenge()
        lg.info("···      𝛃  = %d", beta)
        tr.add_scalar(beta)
    gamma = tr.challenge()
    lg.info("···      𝜸  = %d", gamma)
    lg.info("··· [%s(x)]₁ = %s", sz, _g1_str(C[sz]))
    lg.info("> ROUND 3. Compute the quotient polynomial Q ∈ 𝔽[X]")
    tr.add_scalar(gamma)
    tr.add_commitment(C[sz])
    alpha = tr.challenge()
    lg.info("···      𝜶  = %d", alpha)
    lg.info("··· [Q(x)]₁ = %s", _g1_str(C["Q"]))
    lg.info("> ROUND 4. Compute the evaluations of the polynomials")
    tr.add_scalar(alpha)
    tr.add_commitment(C["Q"])
    xi = tr.challenge()
    lg.info("···      𝔷  = %d", xi)
    evs = []
    for i in range(npols):
        fx = _fr_int(E[f"f{i}xi" if vec else "fxi"])
        lg.info("···   %s  = %d", f"f{i + 1}(𝔷)" if vec else "f(𝔷)", fx)
        evs.append(fx)
        if gs:
            tx = _fr_int(E[f"t{i}xi" if vec else "txi"])
            lg.info("···   %s  = %d", f"t{i + 1}(𝔷)" if vec else "t(𝔷)", tx)
            evs.append(tx)
    if selected:
        evs += [_fr_int(E["selFxi"]), _fr_int(E["selTxi"])]
        lg.info("···   fsel(𝔷)  = %d", evs[-2])
        lg.info("···   tsel(𝔷)  = %d", evs[-1])
    zw = _fr_int(E["sxiw" if gs else "zxiw"])
    lg.info("··· %s(𝔷·𝛚)  = %d", sz, zw)
    lg.info("> ROUND 5. Compute the opening proof polynomials W𝔷, W𝔷𝛚 ∈ 𝔽[X]")
    tr.add_scalar(xi)
    for v in evs + [zw]:
        tr.add_scalar(v)
    v = tr.challenge()
    lg.info("···      v  =  %d", v)
    n = 1 << nbits
    zh = (pow(xi, n, _FR) - 1) % _FR  # polynomial_utils.js:1-19
    l1 = zh * pow(n * (xi - 1) % _FR, _FR - 2, _FR) % _FR
    lg.info("···  ZH(𝔷)  = %d", zh)
    lg.info("···  L₁(𝔷)  = %d", l1)
    lg.info("··· [W𝔷(x)]₁   = %s", _g1_str(C["Wxi"]))
    lg.info("··· [W𝔷·𝛚(x)]₁ = %s", _g1_str(C["Wxiw"]))
    lg.info("")
    lg.info("> MULTISET EQUALITY KZG %s PROVER FINISHED", _TITLE[kind])
    return {"beta": beta, "gamma": gamma, "alpha": alpha, "xi": xi, "v": v}


def grandsum_prover(pTauFilename, evalsFs, evalsTs, evalsSelF=None, evalsSelT=None, device=0):
    """mset_eq_kzg_grandsum_prover (src/grandsum/mset_eq_kzg_prover.js:12)."""
    try:
        return _prover(GRANDSUM, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsSelT, device)
    except KgsError as e:
        raise _semantic(e) from e


def grandproduct_prover(pTauFilename, evalsFs, evalsTs, evalsSelF=None, evalsSelT=None, device=0):
    """mset_eq_kzg_grandproduct_prover (src/grandproduct/mset_eq_kzg_prover.js:12)."""
    try:
        return _prover(GRANDPRODUCT, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsSelT, device)
    except KgsError as e:
        raise _semantic(e) from e


def _verifier(kind, pTauFilename, proof, nBits):
    """src/{grandsum,grandproduct}/mset_eq_kzg_verifier.js:9 — the proof's shape is read from its
    keys as the reference does (nPols from /^F[0-9]/, selectors from /^selF/); the check runs in
    libkgs (kgs_verify_ptau: transcript replay + optimal-ate pairing, host only)."""
    import re
    keys = list(proof["commitments"].keys())
    nfi = len([k for k in keys if re.match(r"^F\d", k)])
    npols = nfi if nfi > 0 else 1
    selected = len([k for k in keys if re.match(r"^selF", k)]) == 1
    if kind == LOOKUP and not selected:
        return False
    cn, en = proof_names(kind, npols, selected)
    try:
        com = b"".join(bytes(proof["commitments"][n]) for n in cn)
        ev = b"".join(bytes(proof["evaluations"][n]) for n in en)
    except KeyError:
        return False
    if len(com) != 64 * len(cn) or len(ev) != 32 * len(en):
        return False
    rc = _check(lib().kgs_verify_ptau(kind, os.fsencode(pTauFilename), nBits, npols, 1 if selected else 0,
                                      _buf(com), _buf(ev)))
    return rc == 1


def grandsum_verifier(pTauFilename, proof, nBits):
    """mset_eq_kzg_grandsum_verifier (src/grandsum/mset_eq_kzg_verifier.js:9)."""
    return _verifier(GRANDSUM, pTauFilename, proof, nBits)


def grandproduct_verifier(pTauFilename, proof, nBits):
    """mset_eq_kzg_grandproduct_verifier (src/grandproduct/mset_eq_kzg_verifier.js:9)."""
    return _verifier(GRANDPRODUCT, pTauFilename, proof, nBits)


def lookup_prover(pTauFilename, evalsFs, evalsTs, evalsSelF=None, evalsMulT=None, device=0):
    """Lookup argument: every selected f row (evalsSelF, binary; all ones if None)
    is a row of the table t, and evalsMulT (Montgomery, required) holds how often each table row is
    looked up. The commented-out cases of test/lookup_kzg_grandsum.test.js:24-44 call the grand-sum
    prover with these arguments; this is that prover without the binary constraint on the
    multiplicities (include/kgs.h KGS_LOOKUP). Same proof layout as a selected grand-sum."""
    try:
        return _prover(LOOKUP, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsMulT, device)
    except KgsError as e:
        raise _semantic(e) from e


def lookup_verifier(pTauFilename, proof, nBits):
    """Verifier of lookup_prover's proofs: the grand-sum verifier (src/grandsum/mset_eq_kzg_verifier.js:9)
    without the selT-binary term of r0 (:80-81)."""
    return _verifier(LOOKUP, pTauFilename, proof, nBits)
