"""The N>1 path on CPU (gloo, world size 2): bench.py's sequence sharding + row0-keyed device
noise gives, rank by rank, exactly the rows of a single-process run, and the MAX all-reduce of
the timing works.  The per-rank compute is the oracle fed the device-noise restatement (there is
no GPU here); on the GPU box tests/test_gpu_parity.py::test_row0_makes_noise_shard_invariant
checks the same invariance on the HIP engine."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O

J, T, BATCH, FUT, SEED = 16, 3, 2, 3, 99


def _small_model():
    from skeletondiffusion_amd.skeletons import skeleton as sk

    _, _, adj, types = sk("h36m16")
    cfg = O.release_config(J, types)
    sd = O.synthetic_state_dict(cfg, 1234)
    S, L, U = O.get_cov_from_corr(torch.from_numpy(adj))
    sd.update(O.nonisotropic_buffers(S, L, U, O.beta_schedule("cosine", T)))
    return cfg, sd


def _run_shard(seq0, row0, rows, batch):
    from skeletondiffusion_amd import synthetic

    cfg, sd = _small_model()
    xc = torch.from_numpy(np.stack([synthetic.uniform((J, 96), 10_000 + seq0 + s) for s in range(batch)]))
    start, samp = O.device_noise(SEED, row0, rows, T, J, 96)
    bufs = {k: v for k, v in sd.items() if not k.startswith("model.")}
    img, _ = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc)
    return img


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    seq0, row0, rows = bench.shard(rank, BATCH, FUT)
    img = _run_shard(seq0, row0, rows, BATCH)
    parts = [torch.empty_like(img) for _ in range(world)]
    dist.all_gather(parts, img)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((torch.cat(parts).numpy(), float(t)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_sharding_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, tmax = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0
    single = _run_shard(0, 0, 2 * BATCH * FUT, 2 * BATCH).numpy()
    # torch-CPU GEMM blocking depends on the batch size, so the oracle is row-invariant only to
    # rounding; the HIP engine is row-invariant bitwise (tested on the GPU box)
    np.testing.assert_allclose(gathered, single, atol=1e-6, rtol=0)


# ---- skeletondiffusion_amd.sharded: broadcast / ragged gather / metric all_reduce (gloo) ----------

NSEQ3, FUT3 = 5, 2  # 5 sequences over 3 ranks: shards of 2, 2, 1 (ragged gather)


def _oracle_sample_fn(x_cond, batch_size, seed, row0):
    """Test stand-in for diffusion.sample on CPU: the oracle fed the device-noise restatement."""
    cfg, sd = _small_model()
    start, samp = O.device_noise(seed, row0, batch_size, T, J, 96)
    bufs = {k: v for k, v in sd.items() if not k.startswith("model.")}
    img, _ = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=x_cond)
    return img


def _sharded_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from skeletondiffusion_amd import sharded, synthetic

    # broadcast_state: every rank ends with rank 0's parameters
    m = torch.nn.Linear(4, 3)
    with torch.no_grad():
        m.weight.fill_(float(rank))
        m.bias.fill_(float(rank) + 0.5)
    sharded.broadcast_state(m)
    ok_bcast = bool((m.weight == 0).all() and (m.bias == 0.5).all())
    xc = torch.from_numpy(np.stack([synthetic.uniform((J, 96), 10_000 + s) for s in range(NSEQ3)]))

    def fn(**kw):
        return _oracle_sample_fn(**kw)

    full, s0 = sharded.sample_sharded(fn, xc, FUT3, SEED)
    local, s0b = sharded.sample_sharded(fn, xc, FUT3, SEED, gather=False)
    per_seq = local.reshape(-1, FUT3, J * 96).abs().mean((1, 2))  # a per-sequence statistic
    mean = sharded.reduce_metric(per_seq, nseq_total=NSEQ3)
    if rank == 0:
        q.put((full.numpy(), float(mean), ok_bcast, s0, s0b))
    else:
        q.put(("rank", rank, ok_bcast, local.shape[0], s0))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_balanced_and_ragged():
    from skeletondiffusion_amd.sharded import shard_range

    assert [shard_range(11015, r, 8) for r in (0, 6, 7)] == [(0, 1377), (8262, 9639), (9639, 11015)]
    for nseq, world in ((5, 3), (2, 4), (16, 8)):
        spans = [shard_range(nseq, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == nseq
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_three_rank_sharded_eval_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(3)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = [g for g in got if not isinstance(g[0], str)][0]
    others = [g for g in got if isinstance(g[0], str)]
    full, mean, ok0, s0, s0b = r0
    assert ok0 and all(o[2] for o in others)
    assert sorted((o[1], o[3], o[4]) for o in others) == [(1, 4, 2), (2, 2, 4)]  # rows, first sequence
    from skeletondiffusion_amd import synthetic

    xc = torch.from_numpy(np.stack([synthetic.uniform((J, 96), 10_000 + s) for s in range(NSEQ3)]))
    single = _oracle_sample_fn(xc, NSEQ3 * FUT3, SEED, 0)
    np.testing.assert_allclose(full, single.numpy(), atol=1e-6, rtol=0)
    ref_mean = single.reshape(NSEQ3, FUT3, J * 96).abs().mean((1, 2)).double().mean().item()
    assert abs(mean - ref_mean) < 1e-6


def _empty_shard_worker(rank, world, port, q):
    """3 ranks, 2 sequences: rank 2 owns no sequence.  Its sample_fn must not be called (the HIP
    engine rejects x_cond with 0 rows, base.py:246-248 semantics), yet it joins the all_gather."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from skeletondiffusion_amd import sharded, synthetic

    xc = torch.from_numpy(np.stack([synthetic.uniform((J, 96), 10_000 + s) for s in range(2)]))
    calls = []

    def fn(batch_size, x_cond, seed, row0):
        if x_cond.shape[0] == 0 or batch_size == 0:
            raise ValueError("x_cond rows (0) must divide the batch")  # what the engine raises
        calls.append(batch_size)
        return _oracle_sample_fn(x_cond, batch_size, seed, row0)

    full, s0 = sharded.sample_sharded(fn, xc, FUT3, SEED)
    q.put((rank, full.numpy(), s0, calls))
    dist.barrier()
    dist.destroy_process_group()


def test_more_ranks_than_sequences():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_shard_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=300) for _ in range(3)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [g[3] for g in got] == [[FUT3], [FUT3], []]
    from skeletondiffusion_amd import synthetic

    xc = torch.from_numpy(np.stack([synthetic.uniform((J, 96), 10_000 + s) for s in range(2)]))
    single = _oracle_sample_fn(xc, 2 * FUT3, SEED, 0).numpy()
    for g in got:
        assert g[1].shape == single.shape
        np.testing.assert_allclose(g[1], single, atol=1e-6, rtol=0)
