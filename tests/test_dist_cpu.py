"""Multi-process (gloo, world_size 2) checks of the image sharding and record gather."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mlic_amd import dist as mdist


def test_lpt_shard_balances_and_covers():
    sizes = [(2176, 3840)] * 2 + [(1088, 1920)] * 6 + [(512, 768)] * 8
    shards = mdist.lpt_shard(sizes, 4)
    assert sorted(i for s in shards for i in s) == list(range(len(sizes)))
    loads = [sum(mdist.padded_pixels(*sizes[i]) for i in s) for s in shards]
    assert max(loads) - min(loads) <= mdist.padded_pixels(1088, 1920)
    assert mdist.lpt_shard(sizes, 4) == shards  # deterministic


def test_group_shard_whole_batches():
    """BASELINE config 4 at 8 ranks: 144 equal jobs in 12 (weight set, shape) groups -> 18 jobs per
    rank in at most 3 batches (LPT would deal every rank 1-3 images of up to 12 groups)."""
    keys = [(r, H, W) for r in range(6) for (H, W) in [(512, 768)] * 20 + [(768, 512)] * 4]
    sizes = [(k[1], k[2]) for k in keys]
    for world in (1, 2, 3, 4, 8):
        shards = mdist.group_shard(keys, sizes, world)
        assert sorted(i for s in shards for i in s) == list(range(len(keys)))
        counts = [len(s) for s in shards]
        assert max(counts) - min(counts) <= 1, counts
        assert all(len({keys[i] for i in s}) <= -(-12 // world) + 2 for s in shards)
        if world == 8:
            assert all(len({keys[i] for i in s}) <= 3 for s in shards)
        assert mdist.group_shard(keys, sizes, world) == shards
    mixed = [(2176, 3840)] * 2 + [(1088, 1920)] * 6
    shards = mdist.group_shard([s for s in mixed], mixed, 2)
    loads = [sum(mdist.padded_pixels(*mixed[i]) for i in s) for s in shards]
    assert max(loads) - min(loads) <= mdist.padded_pixels(2176, 3840)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, njobs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = [(64 * (1 + j % 3), 64 * (2 + j % 2)) for j in range(njobs)]
    mine = mdist.lpt_shard(sizes, world)[rank]
    rec = torch.zeros(len(mine), mdist.RECORD_LEN, dtype=torch.float64)
    for k, j in enumerate(mine):
        rec[k, 0] = j
        rec[k, 1], rec[k, 2] = sizes[j]
        rec[k, 8] = 30.0 + j  # "psnr"
    allrec = mdist.gather_records(rec, max_per_rank=njobs)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
    if rank == 0:
        q.put((allrec.tolist(), float(t)))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_records_world2():
    world, njobs = 2, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, njobs, q)) for r in range(world)]
    for p in procs:
        p.start()
    rows, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert tmax == 2.0
    assert [int(r[0]) for r in rows] == list(range(njobs))
    assert all(abs(r[8] - (30.0 + r[0])) < 1e-9 for r in rows)


def _sweep_worker(rank, world, port, q):
    import argparse
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a = argparse.Namespace(config="kodak-sweep", rate=1, batch=0)
    jobs, total = bench.build_jobs(a, rank, world)
    F = {k: i for i, k in enumerate(mdist.RECORD_FIELDS)}
    rec = torch.zeros(len(jobs), mdist.RECORD_LEN, dtype=torch.float64)
    for k, j in enumerate(jobs):
        rec[k, F["job"]], rec[k, F["H"]], rec[k, F["W"]], rec[k, F["level"]] = j.id, j.H, j.W, j.level
        rec[k, F["bpp_lik"]] = 0.1 * (1 + j.level)
        rec[k, F["psnr"]] = 30.0 + j.id
    mx = torch.tensor([len(jobs)])
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    allrec = mdist.gather_records(rec, max_per_rank=int(mx))
    n_batches = len(bench.batches(jobs))
    if rank == 0:
        q.put((allrec.tolist(), total, [len(jobs)], n_batches))
    else:
        q.put((None, total, [len(jobs)], n_batches))
    dist.barrier()
    dist.destroy_process_group()


def test_kodak_sweep_sharded_world2():
    """BASELINE config 4's job list (24 Kodak-size images incl. 4 portrait x 6 lambda stand-ins = 144
    jobs) sharded by bench.py over 2 ranks in whole (weight set, shape) batches; the gathered records are
    complete and sorted."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rows = next(g[0] for g in got if g[0] is not None)
    assert all(g[1] == 144 for g in got)
    counts = sorted(g[2][0] for g in got)
    assert sum(counts) == 144 and counts[1] - counts[0] <= 1  # equal-pixel jobs: balanced to one job
    assert all(g[3] <= 7 for g in got)  # each rank runs a few whole batches
    assert [int(r[0]) for r in rows] == list(range(144))
    for r in rows:
        j = int(r[0])
        assert int(r[3]) == j // 24  # lambda level
        assert (int(r[1]), int(r[2])) == ((512, 768) if j % 24 < 20 else (768, 512))


def test_request_streams_cover_the_batch():
    """bench.py --split: the main config's 32 images per rank become 4 request streams of 8 (each its
    own model instance at run time), every job exactly once; the VBR config's two batches become 4
    streams; split 1 keeps one batch per (weights, shape)."""
    import argparse
    import bench
    for world, rank in ((1, 0), (8, 3)):
        a = argparse.Namespace(config="main", rate=1, batch=0)
        jobs, total = bench.build_jobs(a, rank, world)
        assert total == 32 * world and len(jobs) == 32
        for split, want in ((4, [8, 8, 8, 8]), (1, [32]), (3, [11, 11, 10])):
            groups = bench.batches(jobs, split=split)
            assert [len(js) for _, js in groups] == want
            ids = sorted(j.id for _, js in groups for j in js)
            assert ids == sorted(j.id for j in jobs)
    a = argparse.Namespace(config="vbr-mixed", rate=1, batch=0)
    jobs, _ = bench.build_jobs(a, 0, 1)
    groups = bench.batches(jobs, split=bench.WORKLOADS["vbr-mixed"]["split"])
    assert sorted(len(js) for _, js in groups) == [1, 1, 3, 3]
    assert sorted(j.id for _, js in groups for j in js) == sorted(j.id for j in jobs)


def _bench_path_worker(rank, world, port, q):
    """bench.main()'s distributed skeleton on gloo: the timed region (barriers, device syncs, elapsed
    max over ranks), the record build for this rank's share of the main config's job list, and the
    gather with its every-job-exactly-once assert -- the same functions main() calls on RCCL."""
    import time
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    a = bench.parse(["--config", "main", "--gpus", str(world), "--steps", "2", "--warmup", "0"])
    jobs, total = bench.build_jobs(a, rank, world)
    groups = bench.batches(jobs, split=a.split)
    ran = []

    def run_steps(n):  # rank 1 is the slow one: the reported time must be its time
        for _ in range(n):
            for gi, (_, js) in enumerate(groups):
                ran.append((gi, len(js)))
            time.sleep(0.05 * (rank + 1))
    syncs = []
    elapsed = bench.timed_steps(run_steps, a.steps, True, dev, sync=lambda: syncs.append(1))
    F = {k: i for i, k in enumerate(mdist.RECORD_FIELDS)}
    rec = torch.zeros(len(jobs), mdist.RECORD_LEN, dtype=torch.float64)
    for k, j in enumerate(jobs):
        rec[k, F["job"]], rec[k, F["H"]], rec[k, F["W"]] = j.id, j.H, j.W
        rec[k, F["psnr"]] = 20.0 + j.id
    allrec = bench.gather_all(rec, total, True, dev)
    # a rank that lost one record: the assert fires on every rank (after the collectives, no hang)
    lost = None
    try:
        bench.gather_all(rec[1:] if rank == 1 else rec, total, True, dev)
    except AssertionError as e:
        lost = str(e)
    q.put((rank, elapsed, len(syncs), len(ran), total, allrec.tolist() if rank == 0 else None, lost))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_distributed_path_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_path_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=180) for _ in range(world)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    el = [g[1] for g in got]
    assert el[0] == el[1] and el[0] >= 2 * 0.1, el  # max over ranks: the slow rank's 2 x 0.1 s
    assert all(g[2] == 4 for g in got)  # device sync twice on each side of the timed steps
    assert all(g[3] == 2 * 4 for g in got)  # 2 steps x the 4 request streams of 8
    assert all(g[4] == 64 for g in got)
    rows = got[0][5]
    assert [int(r[0]) for r in rows] == list(range(64))
    assert all(abs(r[8] - (20.0 + r[0])) < 1e-9 for r in rows)
    assert all(g[6] is not None for g in got)  # a lost record is caught on both ranks
