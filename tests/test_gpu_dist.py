"""GPU tests of the distributed prover (kgs_ctx_set_group): every vector of
the proof sharded over W ranks — NTTs as local transforms + one all-to-all, the builder scan, the
quotient, Horner, the synthetic divisions and every MSM on per-rank slices. On the one-GPU box the
ranks are W contexts on cuda:0 (in-process group, one host thread per rank), or W processes with a
gloo host group, or one process with a world-1 RCCL communicator (the RCCL transport end to end).
Every rank's proof must be byte-identical to the single-GPU prover's (itself pinned to the oracle:
tests/test_gpu_parity.py), and the reference's failure messages must come out of every rank.
"""
import os
import threading

import pytest

import common
from oracle import protocol as P
from test_gpu_configs import gpu_ptau, np_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    return common.load_pkg()


def single(K, ptau, kind, nbits, Fs, Ts, sF, sT):
    ctx = K.Context(0)
    ctx.load_ptau(ptau, nbits)
    out = ctx.prove(kind, nbits, Fs, Ts, sF, sT, mont_out=False)[:2]
    ctx.close()
    return out


def run_group(K, group, world, ptau, kind, nbits, Fs, Ts, sF, sT, mont_out=False, sliced=False, ctxs=None,
              keep=False):
    """one proof over `world` contexts on cuda:0 (one host thread per rank); sliced: every rank
    loads only its SRS slice (kgs_srs_load_ptau_slice), otherwise the whole SRS"""
    own = ctxs is None
    if own:
        ctxs = [K.Context(0) for _ in range(world)]
        for r, c in enumerate(ctxs):
            c.load_ptau(ptau, nbits, slice=(r, world) if sliced else None)
    for r, c in enumerate(ctxs):
        c.set_group(group, r)
    out, err = [None] * world, [None] * world

    def run(r):
        try:
            res = ctxs[r].prove(kind, nbits, Fs, Ts, sF, sT, mont_out=mont_out)
            out[r] = res if mont_out else res[:2]
        except Exception as e:
            err[r] = e
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    for c in ctxs:
        c.set_group(None)
        if own and not keep:
            c.close()
    return out, err


CASES = [  # (world, kind, nbits, npols, selected)
    (1, 0, 5, 1, False), (2, 0, 5, 1, False), (2, 1, 6, 2, True), (4, 0, 9, 1, True), (4, 1, 9, 1, False),
    (8, 0, 7, 1, False), (8, 1, 8, 3, True), (8, 0, 11, 2, True), (8, 1, 12, 1, False), (4, 0, 16, 1, False),
    (2, 1, 14, 1, True), (8, 0, 16, 3, False),
]


@pytest.mark.parametrize("world,kind,nbits,npols,sel", CASES)
def test_local_group_equals_single_gpu(K, world, kind, nbits, npols, sel):
    ptau = gpu_ptau(K, max(nbits, 9))
    Fs, Ts, sF, sT = common.make_inputs(9000 + 31 * world + nbits + npols, nbits, npols, sel)
    want = single(K, ptau, kind, nbits, Fs, Ts, sF, sT)
    g = K.Group.local(world)
    got, err = run_group(K, g, world, ptau, kind, nbits, Fs, Ts, sF, sT)
    g.close()
    assert not any(err), err
    for r in range(world):
        assert got[r] == want, r


SLICED = [(2, 0, 5, 1, False), (4, 1, 9, 2, True), (8, 0, 11, 3, True), (8, 1, 12, 1, False), (4, 0, 16, 1, False)]


@pytest.mark.parametrize("world,kind,nbits,npols,sel", SLICED)
def test_sliced_srs_group_equals_single_gpu(K, world, kind, nbits, npols, sel):
    """every rank holds only its SRS slice (points r + W j): the proof is still byte-identical"""
    ptau = gpu_ptau(K, max(nbits, 9))
    Fs, Ts, sF, sT = common.make_inputs(7000 + 31 * world + nbits + npols, nbits, npols, sel)
    want = single(K, ptau, kind, nbits, Fs, Ts, sF, sT)
    g = K.Group.local(world)
    got, err = run_group(K, g, world, ptau, kind, nbits, Fs, Ts, sF, sT, sliced=True)
    g.close()
    assert not any(err), err
    for r in range(world):
        assert got[r] == want, r


def test_slice_holds_one_wth_of_the_tables(K):
    """kgs_srs_slice_info: a rank's slice is 1/W of the points (and, at the same window, of the bytes);
    a context holding a slice refuses the single-GPU prover"""
    nbits, world = 16, 8
    ptau = gpu_ptau(K, nbits)
    full = K.Context(0)
    full.load_ptau(ptau, nbits)
    _, npts_full, c_full = full.srs_info()
    assert full.srs_slice_info()[:2] == (0, 1)
    full.close()
    for r in (0, 5):
        c = K.Context(0)
        c.load_ptau(ptau, nbits, slice=(r, world))
        _, npts, cw = c.srs_info()
        rank, w, tbytes = c.srs_slice_info()
        assert (rank, w) == (r, world) and npts == (npts_full - r + world - 1) // world  # points r + W j
        W = (255 + cw - 1) // cw
        assert tbytes == W * npts * 64
        Fs, Ts, sF, sT = common.make_inputs(5, 6, 1, False)
        with pytest.raises(K.KgsError, match="SRS slice"):
            c.prove(K.GRANDSUM, 6, Fs, Ts, sF, sT, mont_out=False)
        c.close()


def test_rank_local_failure_is_agreed(K):
    """a precondition that fails on ONE rank (no SRS / another rank's slice) fails every rank at once
    with that rank's error, before any exchange; the group stays usable"""
    world, nbits = 4, 9
    ptau = gpu_ptau(K, 9)
    Fs, Ts, sF, sT = common.make_inputs(99, nbits, 1, False)
    want = single(K, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    g = K.Group.local(world)
    ctxs = [K.Context(0) for _ in range(world)]
    for r, c in enumerate(ctxs):
        if r != 2:
            c.load_ptau(ptau, nbits, slice=(r, world))
    _, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT, ctxs=ctxs)
    assert all(isinstance(e, K.KgsError) and "no SRS loaded" in str(e) for e in err), err
    ctxs[2].load_ptau(ptau, nbits, slice=(1, world))  # the wrong slice
    _, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT, ctxs=ctxs)
    assert all(isinstance(e, K.KgsError) and "is not this context's" in str(e) for e in err), err
    ctxs[2].load_ptau(ptau, nbits, slice=(2, world))
    got, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT, ctxs=ctxs)
    assert not any(err), err
    assert all(x == want for x in got)
    for c in ctxs:
        c.close()
    g.close()


@pytest.mark.parametrize("world,nbits,npols,sel", [(8, 20, 1, False), (4, 22, 2, True)])
def test_local_group_large(K, world, nbits, npols, sel):
    """configs[3]/[4]-style shapes on one GPU: sharded == unsharded, and the proof verifies"""
    ptau = gpu_ptau(K, nbits)
    Fs, Ts, sF, sT = np_inputs(0xD157 + world, nbits, npols, sel)
    want = single(K, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    g = K.Group.local(world)
    got, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    g.close()
    assert not any(err), err
    assert all(x == want for x in got)
    cn, en = K.proof_names(K.GRANDSUM, npols, sel)
    assert K.grandsum_verifier(ptau, {"commitments": dict(zip(cn, want[0])), "evaluations": dict(zip(en, want[1]))},
                               nbits) is True


def test_dist_montgomery_writeback(K):
    """the drop-in host path under the group: every rank writes the caller's Montgomery forms back"""
    world, nbits = 4, 9
    ptau = gpu_ptau(K, 9)
    Fs, Ts, sF, sT = common.make_inputs(4321, nbits, 2, False)
    g = K.Group.local(world)
    got, err = run_group(K, g, world, ptau, K.GRANDPRODUCT, nbits, Fs, Ts, sF, sT, mont_out=True)
    g.close()
    assert not any(err), err
    want_mf = [common.mont_bytes([int.from_bytes(f[32 * j:32 * j + 32], "little") for j in range(1 << nbits)])
               for f in Fs]
    for r in range(world):
        assert [bytes(x) for x in got[r][2]] == want_mf


def test_dist_error_messages(K):
    """the reference's failures come out of every rank, and the group stays usable afterwards"""
    world, nbits = 4, 9
    ptau = gpu_ptau(K, 9)
    g = K.Group.local(world)
    Fs, _, _, _ = common.make_inputs(1, nbits, 1, False)
    F2, _, _, _ = common.make_inputs(2, nbits, 1, False)
    _, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, F2, None, None)
    assert all(isinstance(e, K.KgsError) and str(e) == "The grand-sum polynomial S is not well calculated" for e in err)
    _, err = run_group(K, g, world, ptau, K.GRANDPRODUCT, nbits, Fs, F2, None, None)
    assert all(str(e) == "The grand-product polynomial Z is not well calculated" for e in err)
    # a selector that is not binary: the quotient numerator is not divisible by Z_H
    Fs, Ts, sF, sT = common.make_inputs(3, nbits, 1, True)
    sF = common.mont_bytes([2] + [1] * ((1 << nbits) - 1))
    _, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    want = single_err(K, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    assert all(str(e) == want for e in err), (err, want)
    # still usable
    Fs, Ts, sF, sT = common.make_inputs(4, nbits, 1, False)
    got, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    assert not any(err) and all(x == single(K, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT) for x in got)
    g.close()


def single_err(K, ptau, kind, nbits, Fs, Ts, sF, sT):
    ctx = K.Context(0)
    ctx.load_ptau(ptau, nbits)
    try:
        ctx.prove(kind, nbits, Fs, Ts, sF, sT, mont_out=False)
    except K.KgsError as e:
        return str(e)
    finally:
        ctx.close()
    return None


def test_rccl_transport_world1(K):
    """the RCCL group (grouped ncclSend/ncclRecv all-to-all on the prover stream, ncclAllGather for
    the small exchanges) driving the distributed prover with a one-rank communicator"""
    nbits = 10
    ptau = gpu_ptau(K, 10)
    Fs, Ts, sF, sT = common.make_inputs(777, nbits, 2, True)
    want = single(K, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    g = K.Group.rccl(0, 1, K.rccl_unique_id(), 0)
    got, err = run_group(K, g, 1, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    g.close()
    assert not any(err), err
    assert got[0] == want


def _gloo_dist_rank(rank, world, port, ptau, q, a2a):
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        K = common.load_pkg()
        ctx = K.Context(0)
        ctx.load_ptau(ptau, 10)
        g = K.Group.host(world, K.torch_allgather(), K.torch_alltoall() if a2a else None)
        ctx.set_group(g, rank)
        Fs, Ts, sF, sT = common.make_inputs(2718, 10, 2, True)
        coms, evs = ctx.prove(K.GRANDPRODUCT, 10, Fs, Ts, sF, sT, mont_out=False)[:2]
        x = ctx.last_exchange()
        # the transport's own bytes: without the all-to-all callback every rank all-gathers its whole
        # send buffer, W times the all-to-all model's
        model = K.dist_exchange_model(K.GRANDPRODUCT, 10, 2, True, world)["alltoall_bytes"]
        if x["alltoall_bytes"] != (model if a2a else model * world):
            coms, evs = None, f"exchange bytes {x}"
        ctx.set_group(None)
        ctx.close()
        g.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, coms, evs))
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("a2a", [False, True])
def test_host_group_two_processes(K, a2a):
    """one process per rank (as under torchrun) with the distributed prover over a gloo host group:
    all-gather only, and with the all-to-all callback (torch all_to_all_single: (W - 1) / W of a
    vector leaves a rank per exchange)"""
    import multiprocessing as mp
    import socket
    ptau = gpu_ptau(K, 10)
    Fs, Ts, sF, sT = common.make_inputs(2718, 10, 2, True)
    want = single(K, ptau, K.GRANDPRODUCT, 10, Fs, Ts, sF, sT)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    procs = [mpc.Process(target=_gloo_dist_rank, args=(r, 2, port, ptau, q, a2a)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, coms, evs in res:
        assert coms is not None, evs
        assert (coms, evs) == want, rank


@pytest.mark.parametrize("world,kind,nbits,npols,sel", [(2, 0, 10, 1, False), (4, 1, 10, 2, True), (8, 1, 9, 1, False)])
def test_exchange_stats_match_the_model(K, world, kind, nbits, npols, sel):
    """kgs_last_exchange on every rank: the all-to-all count and the bytes that left the rank are
    those of K.dist_exchange_model (the DESIGN.md §6 plan the bench's exchange fields are read
    against); the spans are positive; a single-GPU proof afterwards reports zeros"""
    ptau = gpu_ptau(K, 12)
    Fs, Ts, sF, sT = common.make_inputs(99, nbits, npols, sel)
    g = K.Group.local(world)
    ctxs = [K.Context(0) for _ in range(world)]
    for c in ctxs:
        c.load_ptau(ptau, nbits)
    got, err = run_group(K, g, world, ptau, kind, nbits, Fs, Ts, sF, sT, ctxs=ctxs, keep=True)
    assert not any(err), err
    model = K.dist_exchange_model(kind, nbits, npols, sel, world)
    for c in ctxs:
        x = c.last_exchange()
        assert x["alltoall_n"] == model["alltoall_n"] and x["alltoall_bytes"] == model["alltoall_bytes"], (x, model)
        assert x["alltoall_ms"] > 0 and x["allgather_n"] > 0 and x["allgather_bytes"] > 0
    ctxs[0].prove(kind, nbits, Fs, Ts, sF, sT, mont_out=False)
    assert ctxs[0].last_exchange()["alltoall_n"] == 0
    for c in ctxs:
        c.close()
    g.close()


def test_dist_matches_oracle_small(K):
    """one small distributed case checked directly against the CPU oracle as well"""
    nbits, world = 7, 8
    ptau = common.oracle_ptau(9)
    srs = P.SRS(ptau, common.tau())
    Fs, Ts, sF, sT = common.make_inputs(55, nbits, 1, True)
    g = K.Group.local(world)
    got, err = run_group(K, g, world, ptau, K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    g.close()
    assert not any(err), err
    exp = P.prove("grandsum", srs, P.EvalBuffer(Fs[0]), P.EvalBuffer(Ts[0]), P.EvalBuffer(sF), P.EvalBuffer(sT))
    cn, en = K.proof_names(K.GRANDSUM, 1, True)
    assert got[0] == ([exp["commitments"][c] for c in cn], [exp["evaluations"][e] for e in en])
