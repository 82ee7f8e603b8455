"""Multi-GPU path on CPU: MSM point-range sharding (include/kgs.h kgs_ctx_set_shard).

The sharded prover cuts every commitment MSM into `world` contiguous point ranges
(kgs_shard_range), runs Pippenger per rank and all-gathers the per-rank bit-sum partials
(c XYZZ points T_k) once per prover round; every rank then combines them with kgs_msm_combine.
Here (no GPU) the decomposition, the torch.distributed transport (gloo, world_size 2) and the
product's host combiner are checked against the oracle's MSM (oracle/bn254.py); the full sharded
prover is checked on the GPU in test_gpu_parity.py (test_sharded_prover_*).
"""
import multiprocessing as mp
import os
import random
import socket
import sys

import pytest

import common
from oracle import bn254 as O


def xyzz_bytes(p):
    """affine oracle point -> 128 B XYZZ (X, Y, ZZ = ZZZ = 1; LE Montgomery Fq); None -> zeros."""
    if p is None:
        return bytes(128)
    one = O.fq_to_bytes(1)
    return O.fq_to_bytes(p[0]) + O.fq_to_bytes(p[1]) + one + one


def partial_from_point(p, c):
    """a valid rank partial: T_0 = p, T_k = infinity for k > 0"""
    return xyzz_bytes(p) + bytes(128 * (c - 1))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(world):
    K = common.load_pkg()
    for n in (0, 1, 7, 8, 1000, (1 << 20) - 2, (1 << 24) + 5):
        ranges = [K.shard_range(n, r, world) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        for (a, b), (c, d) in zip(ranges, ranges[1:]):
            assert b == c and a <= b
        sizes = [b - a for a, b in ranges]
        assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_rank():
    K = common.load_pkg()
    with pytest.raises(K.KgsError):
        K.shard_range(10, 2, 2)


@pytest.mark.parametrize("nparts,c", [(1, 6), (2, 8), (8, 16)])
def test_msm_combine_matches_oracle(nparts, c):
    K = common.load_pkg()
    rng = random.Random(1000 * nparts + c)
    T = b""
    total = 0
    for _ in range(nparts):
        for k in range(c):
            if rng.random() < 0.2:
                T += bytes(128)  # infinity partial
                continue
            a = rng.randrange(1, O.R)
            total += a << k
            T += xyzz_bytes(O.g1_mul(O.G1_GEN, a))
    got = K.msm_combine(T, nparts, c)
    assert got == O.g1_to_lem(O.g1_mul(O.G1_GEN, total % O.R))


def test_msm_combine_all_infinity():
    K = common.load_pkg()
    assert K.msm_combine(bytes(2 * 4 * 128), 2, 4) == bytes(64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_rank(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, common.ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        K = common.load_pkg()
        rng = random.Random(7)  # same points/scalars on every rank (replicated inputs)
        N, c = 37, 8
        pts = [O.g1_mul(O.G1_GEN, rng.randrange(1, O.R)) for _ in range(N)]
        sc = [rng.randrange(0, O.R) for _ in range(N)]
        lo, hi = K.shard_range(N, rank, world)
        mine = O.g1_sum([O.g1_mul(p, s) for p, s in zip(pts[lo:hi], sc[lo:hi])])
        gather = K.torch_allgather()
        # two commitments in one exchange, as the prover batches a round
        send = partial_from_point(mine, c) + partial_from_point(O.g1_neg(mine) if mine else None, c)
        recv = gather(send)
        assert len(recv) == world * len(send)
        tb = 128 * c
        parts1 = b"".join(recv[r * len(send): r * len(send) + tb] for r in range(world))
        parts2 = b"".join(recv[r * len(send) + tb: (r + 1) * len(send)] for r in range(world))
        full = O.g1_sum([O.g1_mul(p, s) for p, s in zip(pts, sc)])
        ok1 = K.msm_combine(parts1, world, c) == O.g1_to_lem(full)
        ok2 = K.msm_combine(parts2, world, c) == O.g1_to_lem(O.g1_neg(full) if full else None)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok1 and ok2, (lo, hi)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_msm(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    ranges = sorted(r[2] for r in res)
    assert ranges[0][0] == 0 and ranges[-1][1] == 37


def _a2a_rank(rank, world, port, q):
    try:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, common.ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        K = common.load_pkg()
        chunk = 96

        def block(src, dst):
            return bytes((31 * src + 7 * dst + i) % 256 for i in range(chunk))
        send = b"".join(block(rank, j) for j in range(world))  # chunk j goes to rank j
        out = K.torch_alltoall()(send, chunk)
        ok = out == b"".join(block(s, rank) for s in range(world))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok, len(out)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_alltoall_transport(world):
    """K.torch_alltoall (the host group's all-to-all callback, kgs_group_create_host_a2a): chunk j
    of every rank's buffer reaches rank j, in source-rank order; a rank receives world chunks (one
    vector), not world x its vector as through the all-gather-only transport"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(n == 96 * world for _, _, n in res)


def test_dist_exchange_model():
    """The all-to-alls of one distributed proof (csrc/prover_dist.cpp): a grand-sum
    with k = 1 moves 12 vectors, 6 of length n and 6 of the 2n coset, i.e. 18 n-vector
    equivalents, each sending L / W^2 elements to each of the W - 1 other ranks; selectors add two
    of each; a vector adds two n-vectors per extra multiset; the unselected grand-product's coset
    has n points. At n = 2^24 over 8 ranks that is 1.06 GB per rank (~1.1 GiB)."""
    K = common.load_pkg()
    n = 1 << 20
    for W in (2, 4, 8, 16):
        def unit(x):
            return 32 * (W - 1) * x // (W * W)
        m = K.dist_exchange_model(K.GRANDSUM, 20, 1, False, W)
        assert m == {"alltoall_n": 12, "alltoall_bytes": unit(18 * n)}
        m = K.dist_exchange_model(K.GRANDSUM, 20, 1, True, W)
        assert m == {"alltoall_n": 16, "alltoall_bytes": unit(8 * n + 8 * 2 * n)}
        m = K.dist_exchange_model(K.GRANDPRODUCT, 20, 1, False, W)
        assert m == {"alltoall_n": 12, "alltoall_bytes": unit(12 * n)}
        m = K.dist_exchange_model(K.GRANDSUM, 20, 3, False, W)
        assert m == {"alltoall_n": 16, "alltoall_bytes": unit(22 * n)}
        assert K.dist_exchange_model(K.LOOKUP, 20, 1, True, W) == K.dist_exchange_model(K.GRANDSUM, 20, 1, True, W)
    assert K.dist_exchange_model(K.GRANDSUM, 24, 1, False, 8)["alltoall_bytes"] == 1056964608
