"""MLIC++ encode+decode throughput on MI355X (BASELINE.json configs 2-5).

One step = compress() + decompress() (real rANS bitstreams) of every image of the workload on each
GPU.  Images shard across ranks (one process per GPU); the only collective is an all_gather of
fixed-size per-image records after the timed region.

    python bench.py [--config main|kodak|s1080|sd1080|kodak-sweep|vbr-mixed] [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Workloads (weights: seeded realistic-rate sets, mlic_amd/synthetic.py RATE_LAMBDAS; no checkpoints
offline; images: seeded synthetic):
  main        config 2: MLICPP_L, 32 x 1920x1088 per GPU (weak scaling)        <- the default line
  kodak       config 1 shape on the GPU: MLICPP_L, 64 x 768x512 per GPU (weak)
  s1080       config 3: MLICPP_S, 32 x 1920x1088 per GPU (weak)
  sd1080      config 3: MLICPP_M_SMALL_DEC, 32 x 1920x1088 per GPU (weak)
  kodak-sweep config 4: MLICPP_L, 24 Kodak-size images (20 x 768x512 + 4 portrait 512x768) x 6
              lambda stand-ins = 144 jobs, LPT-sharded over the ranks (strong scaling)
  vbr-mixed   config 5: MLICPP_L_VBR, 2 x 3840x2176 + 6 x 1920x1088 per GPU, a VBR level per image
              (weak scaling)
Rank 0 prints ONE JSON line.  `roofline` is the kernel family with the most device time in the timed
configuration, measured live with HIP events on the executor streams in an extra untimed step, plus
`step_frac` = T_roof / T_meas over every kernel of the step; `cpu_baseline` times the
CPU oracle (torch fp32 restatement + native rANS) on a bounded sample on this box's cores.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (enc+dec) at 1920×1088 MLICPP_L, 1/2/4/8 GPU; bpp/PSNR Δ vs ref"
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak (spec)


# dense peak of the arithmetic each kernel family runs on (MI355X_MICROARCH.md): fp32 MFMA 157.3 TF;
# the split-fp16 kernels issue 3 fp16 MFMAs (2.5 PF dense) per fp32 product => 2500/3 TF of
# fp32-equivalent work; the VALU kernels run exact fp32 FMAs (157.3 TF with packed FMA)
def kernel_peak(name: str):
    if name.startswith(("conv_f16x3", "conv_x3v2", "pw_resident", "conv_halo", "conv_x4", "chain_", "dwpw_")):
        return 2500.0 / 3, "3 x fp16 MFMA per fp32 product (split-fp16)"
    if name.startswith("local_attn"):
        return 2500.0 / 3, "3 x fp16 MFMA per fp32 product (split-fp16)"
    if name.startswith("conv_mfma"):
        return 157.3, "v_mfma_f32_32x32x2_f32"
    return 157.3, "fp32 VALU FMA"


def family(cat_name: str) -> str:
    """Kernel family = template name without its <...> instantiation (rocprof lists each one)."""
    return cat_name.split("<")[0]


WORKLOADS = {
    # the 32 images of a step as 4 request streams of 8: a stream's decompress starts as soon as its own
    # compress + rANS encode is done, instead of every lane waiting for the slowest lane's encode
    # (measured 86.9-88.1 img/s against 83.0-85.7 as one 32-image call on 4 lanes).  One lane per stream
    # since round 5 (faster kernels: 101.5-101.7 against 99.7-100.4 with 2 lanes, 94.2 with 3; 8 streams
    # of 4: 96.2-96.3; alternating on one box, profiles/r05/ab/host_schedule_ab.log)
    "main": dict(model="MLICPP_L", groups=[(1088, 1920, 32)], scaling="weak", split=4, lanes=1,
                 desc="config 2: MLICPP_L compress+decompress of 1920x1088 images"),
    "kodak": dict(model="MLICPP_L", groups=[(512, 768, 64)], scaling="weak",
                  desc="config 1 shape on GPU: MLICPP_L compress+decompress of 768x512 (Kodak-size) images"),
    "s1080": dict(model="MLICPP_S", groups=[(1088, 1920, 32)], scaling="weak",
                  desc="config 3: MLICPP_S compress+decompress of 1920x1088 images"),
    # (request streams: sd1080 88.9-89.2 vs 88.0-88.3 img/s; MLICPP_S and the Kodak-size batch do not
    # gain -- 223-227 either way, and 392-405 against 460-462 for Kodak-size)
    "sd1080": dict(model="MLICPP_M_SMALL_DEC", groups=[(1088, 1920, 32)], scaling="weak", split=4, lanes=2,
                   desc="config 3: MLICPP_M_SMALL_DEC compress+decompress of 1920x1088 images"),
    # the sweep's 12 (rate, shape) batches of 4-20 Kodak-size images fill the GPU best as 6 concurrent
    # batches of 1 lane each (round 4, alternating: 425.7 / 428.0 img/s against 308.4 / 325.1 with 2 lanes,
    # 411.9 / 424.0 with 8 x 1); a rank holding a single batch (rank 0 of 8: 18 images) keeps 2 lanes
    # (322.6 / 322.8 against 299.9 with 1)
    "kodak-sweep": dict(model="MLICPP_L", scaling="strong", lanes=2, lanes_many=1, group_concurrency=6,
                        desc="config 4: MLICPP_L 24 Kodak-size images x 6 lambda stand-ins, LPT-sharded"),
    # (4 request streams of 1-3 images: 40.2-40.4 img/s against 39.4-39.6 as two batches; one lane per
    # stream since round 5: 43.3-44.1 against 41.9-42.3 with 2)
    "vbr-mixed": dict(model="MLICPP_L_VBR", groups=[(2176, 3840, 2), (1088, 1920, 6)], scaling="weak", split=2, lanes=1,
                      desc="config 5: MLICPP_L_VBR 4K + 1080p batch, one VBR level per image"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="main", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="override the per-GPU batch of a single-group workload")
    ap.add_argument("--rate", type=int, default=1,
                    help="realistic-rate weight set (0..5, synthetic.RATE_LAMBDAS) of fixed-rate workloads; "
                         "-1 = the round-1 high-rate set")
    ap.add_argument("--lanes", type=int, default=0,
                    help="host threads x HIP streams per GPU for compress/decompress (0: the workload's "
                         "default, else $MLIC_LANES or 4)")
    ap.add_argument("--precision", type=int, default=int(os.environ.get("MLIC_PRECISION", "2")),
                    help="dense-conv arithmetic: 2 = split-fp16 MFMA v2 + specialised kernels, "
                         "1 = f16x3 v1 tiles (A/B library only: make AB=1), 0 = fp32 MFMA")
    ap.add_argument("--synth-fp16", action="store_true",
                    help="SURVEY 8(f)4: g_s subpel convs on fp16 operands with fp32 accumulation (x_hat within "
                         "the 0.01 dB gate, bitstreams unchanged); default off: the headline stays fp32-faithful")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip the profiled passes")
    ap.add_argument("--layers-out", default="", help="write the per-layer timing table here")
    ap.add_argument("--records-out", default="", help="write the gathered per-image records (JSON) here")
    ap.add_argument("--profile-lanes", type=int, default=0,
                    help="lanes of the profiled step (0 = same as --lanes, so its launches match the timed "
                         "steps' and rocprofv3's per-kernel averages; 1 = isolated per-kernel times)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"),
                    help="PMC-derived HBM bytes per launch of the dominant family (tools/pmc_traffic.py)")
    ap.add_argument("--group-concurrency", type=int, default=0,
                    help="(weights, shape) batches of a step run concurrently, each on its own model "
                         "instance, lanes and stream (1 = one after another)")
    ap.add_argument("--split", type=int, default=0,
                    help="cut each (weights, shape) batch into this many request streams, each an independent "
                         "compress -> decompress chain on its own model instance (0: the workload's default)")
    ap.add_argument("--schedule", choices=["join", "streams"], default=os.environ.get("MLIC_SCHEDULE", "streams"),
                    help="join: the batches of a step meet at a join every step; streams: when every batch has "
                         "its own worker, each runs its K steps back to back")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="run rank --emulate-rank's share of a W-rank job list on this one GPU, with 1/W of "
                         "the host cores (a prediction of one rank of a W-GPU run; value = that rank's img/s)")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--phase", choices=["both", "decode"], default="both",
                    help="both: a step = compress + decompress (the metric's enc+dec); decode: a step = "
                         "decompress() of streams encoded before the timed region (north_star's decode target)")
    ap.add_argument("--no-decode-record", action="store_true",
                    help="phase both: skip the decode sub-record (a second timed region of K decompress-only "
                         "steps over the streams the timed enc+dec steps produced, with its own roofline)")
    a = ap.parse_args(argv)
    wl = WORKLOADS[a.config]
    a.lanes_auto = a.lanes <= 0 and "MLIC_LANES" not in os.environ and "lanes_many" in wl
    if a.lanes <= 0:
        a.lanes = int(os.environ["MLIC_LANES"]) if "MLIC_LANES" in os.environ else wl.get("lanes", 4)
    if a.group_concurrency <= 0:
        a.group_concurrency = wl.get("group_concurrency", 4)
    if a.split <= 0:
        a.split = wl.get("split", 1)
    return a


# ------------------------------------------------------------------------------------------ jobs
class Job:
    __slots__ = ("id", "model", "rate", "H", "W", "seed", "level")

    def __init__(self, id, model, rate, H, W, seed, level=-1):
        self.id, self.model, self.rate, self.H, self.W, self.seed, self.level = id, model, rate, H, W, seed, level


def build_jobs(a, rank: int, world: int):
    """This rank's jobs and the global job count."""
    from mlic_amd import dist as mdist
    wl = WORKLOADS[a.config]
    rate = None if a.rate < 0 else a.rate
    if a.config == "kodak-sweep":
        # 24 Kodak-size images (the set has 4 portrait members) x 6 weight sets = 144 jobs,
        # cut into contiguous runs of (weight set, shape) batches: whole batches per rank
        shapes = [(512, 768)] * 20 + [(768, 512)] * 4
        alljobs = [Job(r * 24 + i, wl["model"], r, H, W, 2000 + i, r) for r in range(6) for i, (H, W) in enumerate(shapes)]
        mine = mdist.group_shard([(j.rate, j.H, j.W) for j in alljobs], [(j.H, j.W) for j in alljobs], world)[rank]
        return [alljobs[i] for i in mine], len(alljobs)
    groups = wl["groups"]
    if a.batch > 0 and len(groups) == 1:
        groups = [(groups[0][0], groups[0][1], a.batch)]
    per_rank = sum(g[2] for g in groups)
    rng = np.random.Generator(np.random.PCG64(77 + rank))
    jobs, k = [], 0
    vbr = a.config == "vbr-mixed"
    vrate = 2 if rate is None else rate
    for (H, W, n) in groups:
        for _ in range(n):
            level = int(rng.integers(0, 6)) if vbr else (-1 if rate is None else rate)
            jobs.append(Job(rank * per_rank + k, wl["model"], vrate if vbr else rate, H, W, 1000 * rank + k, level))
            k += 1
    return jobs, per_rank * world


def batches(jobs, max_pixels=32 * 1088 * 1920, split=1):
    """Group jobs by (weights, shape) into batches of at most ~32 1080p images' worth of pixels, each
    cut into `split` near-equal request streams."""
    out = {}
    for j in jobs:
        out.setdefault((j.model, j.rate, j.H, j.W), []).append(j)
    res = []
    for key, js in sorted(out.items(), key=lambda kv: (str(kv[0][1]), kv[0][2], kv[0][3])):
        cap = max(1, max_pixels // (key[2] * key[3]))
        cap = min(cap, -(-len(js) // max(1, split)))
        for i in range(0, len(js), cap):
            res.append((key, js[i:i + cap]))
    return res


def psnr_from_mse(mse: float) -> float:
    return 20 * math.log10(255.0) - 10 * math.log10(mse) if mse > 0 else 99.0


def mse_u8(a: torch.Tensor, b: torch.Tensor):
    """utils/utils.py:86-87 (clamp, *255, truncate) + utils/metrics.py:32-33, per image."""
    qa = (a.clamp(0, 1) * 255).to(torch.uint8).float()
    qb = (b.clamp(0, 1) * 255).to(torch.uint8).float()
    return ((qa - qb) ** 2).flatten(1).mean(1).double().cpu().tolist()


# ------------------------------------------------------------------------------------------ CPU side
def _cpu_thread_choice(candidates, probe):
    """Time `probe` (a short slice of the same oracle work) at each thread count; the fastest wins.
    The box's core count is not the box's best thread count: a GPU box may give one GPU's process a
    share of a much larger host, so the choice is measured, not assumed."""
    times = {}
    for n in candidates:
        torch.set_num_threads(n)
        probe()  # warm the thread pool at this size
        t0 = time.perf_counter()
        probe()
        times[n] = time.perf_counter() - t0
    best = min(times, key=times.get)
    return best, {str(k): round(v, 4) for k, v in times.items()}


def cpu_baseline(model: str, rate, H: int, W: int, level: int = -1, phase: str = "both", seed: int = 0):
    """Oracle (torch CPU fp32 restatement of the reference) enc+dec of one image, with the native
    rANS coder for the entropy-coding part, on the best thread count of this box's cores (measured
    over 16 / 32 / 64 / all of this process's affinity on a short g_a probe, then the whole image at that
    count).  Returns the baseline record and the oracle's own coding result of that image (bytes,
    likelihood bpp, x_hat) for the headline's delta (`quality.delta_vs_cpu_oracle`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mlic_ref_cpu as ref
    from mlic_amd import bitstream, entropy, synthetic
    aff = len(os.sched_getaffinity(0))
    total = os.cpu_count() or aff
    sd = synthetic.synth_state_dict(model, 0, rate=rate)
    m = ref.RefMLIC(model, sd)
    x = synthetic.synth_image(H, W, seed)
    s = max(0, level)
    xp = x[:, :, :256, :512].contiguous()
    cands = sorted({c for c in (16, 32, 64, aff) if c <= aff} or {aff})
    threads, probe_s = _cpu_thread_choice(cands, lambda: m.g_a(xp))
    torch.set_num_threads(threads)
    tables = entropy.gaussian_tables(entropy.get_scale_table())
    eb = {k.split(".", 1)[1]: v for k, v in sd.items() if k.startswith("entropy_bottleneck.")}
    etab = entropy.bottleneck_tables(eb)
    t0 = time.time()
    st = m.compress_streams(x, s=s, likelihoods=True)
    sym = torch.cat([p[0].reshape(-1) for p in st["phases"]]).numpy()
    idx = torch.cat([p[1].reshape(-1) for p in st["phases"]]).numpy()
    data = entropy.rans_encode(sym, idx, *tables[:3])
    zs = st["z_symbols"]
    zidx = np.broadcast_to(np.arange(zs.shape[1], dtype=np.int32)[:, None, None], zs.shape[1:]).reshape(-1)
    zdata = entropy.rans_encode(zs.reshape(-1).numpy(), zidx, *etab)
    t1 = time.time()
    dec = entropy.rans_decode(data, idx, *tables[:3])
    zdec = entropy.rans_decode(zdata, zidx, *etab).reshape(zs.shape)
    offs = np.cumsum([0] + [p[0].numel() for p in st["phases"]])
    phase_syms = [torch.from_numpy(dec[offs[k]:offs[k + 1]]).reshape(st["phases"][k][0].shape)
                  for k in range(len(st["phases"]))]
    x_hat = m.decode_streams(torch.from_numpy(zdec), phase_syms, s=s)["x_hat"]
    t2 = time.time()
    dt = (t2 - t1) if phase == "decode" else (t2 - t0)
    lik = st["likelihoods"]
    nbytes = bitstream.file_bytes(len(data), len(zdata), vbr=level >= 0)
    coded = {"bytes": nbytes, "bpp_file": 8.0 * nbytes / (H * W),
             "bpp_lik": ref.bpp_from_likelihoods(lik["y_likelihoods"], lik["z_likelihoods"], H * W),
             "psnr": ref.psnr_uint8(x, x_hat), "H": H, "W": W}
    what = "decoder network + native rANS decode" if phase == "decode" else "encoder+decoder networks + native rANS"
    rec = {"value": round(1.0 / dt, 5), "unit": "images/sec (decode)" if phase == "decode" else "images/sec (enc+dec)",
           "decode_value": round(1.0 / (t2 - t1), 5),
           "cores": threads, "threads_used": threads, "cores_total": total, "cores_affinity": aff,
           "thread_probe_s": probe_s, "kind": "port",
           "sample": f"1 image {W}x{H} {model} (rate set {rate}, seed {seed}: a GPU job's image): oracle torch-CPU fp32 {what}, "
                     f"{dt:.1f} s on {threads} threads (best of {cands} on a g_a probe; {total} host cores, "
                     f"{aff} in this process's affinity)"}
    return rec, coded


def oracle_deltas(model: str, levels, H: int, W: int, gpu_nets, dev):
    """Per-lambda bpp / PSNR delta vs the CPU oracle on one image (kodak-sweep): GPU forward vs oracle."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mlic_ref_cpu as ref
    from mlic_amd import synthetic
    x = synthetic.synth_image(H, W, 2000)
    out = {}
    for r in levels:
        o = ref.RefMLIC(model, synthetic.synth_state_dict(model, rate=r)).forward(x)
        g = gpu_nets[r](x.to(dev))
        bc = ref.bpp_from_likelihoods(o["likelihoods"]["y_likelihoods"], o["likelihoods"]["z_likelihoods"], H * W)
        bg = ref.bpp_from_likelihoods(g["likelihoods"]["y_likelihoods"].cpu(), g["likelihoods"]["z_likelihoods"].cpu(),
                                      H * W)
        pc, pg = ref.psnr_uint8(x, o["x_hat"]), ref.psnr_uint8(x, g["x_hat"].cpu())
        out[f"lambda_{synthetic.RATE_LAMBDAS[r]}"] = {"bpp_gpu": round(bg, 6), "bpp_cpu": round(bc, 6),
                                                      "d_bpp": round(bg - bc, 7), "psnr_gpu": round(pg, 5),
                                                      "psnr_cpu": round(pc, 5), "d_psnr_db": round(pg - pc, 6)}
    return out


# ------------------------------------------------------------------------------- timing + collectives
def timed_steps(run_steps, steps: int, distributed: bool, dev, sync=None) -> float:
    """The timed region: barrier + device sync on both sides of exactly `steps` steps; returns the
    elapsed seconds, max over ranks (all_reduce MAX on `dev`: RCCL on the GPU box, gloo in the CPU
    test).  `sync` is torch.cuda.synchronize on a GPU."""
    sync = sync or (lambda: None)
    sync()
    if distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run_steps(steps)
    sync()
    if distributed:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_all(rec: torch.Tensor, n_expected: int, distributed: bool, dev) -> torch.Tensor:
    """The one data collective: every rank's fixed-size per-image records, all_gathered (padded to the
    largest rank's count, agreed by an all_reduce MAX) and sorted by job; asserts that every job of the
    list is there exactly once."""
    from mlic_amd import dist as mdist
    max_per_rank = max(rec.shape[0], 1)
    if distributed:
        mx = torch.tensor([max_per_rank], device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        max_per_rank = int(mx.item())
    allrec = mdist.gather_records(rec.to(dev), max_per_rank=max_per_rank).cpu()
    ids = allrec[:, 0].long().tolist()
    assert len(ids) == n_expected and len(set(ids)) == n_expected, (len(ids), len(set(ids)), n_expected)
    return allrec


# ------------------------------------------------------------------------------------------ main
def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    emulated = a.emulate_world > 1
    if emulated:
        assert not distributed and 0 <= a.emulate_rank < a.emulate_world, "--emulate-world runs one process"
    # the job list's world / rank, and this process's slot among the node's ranks
    jworld, jrank = (a.emulate_world, a.emulate_rank) if emulated else (world, rank)
    nloc = a.emulate_world if emulated else int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    lslot = a.emulate_rank if emulated else local
    # host cores per rank, before any GPU call: the ranks of a node split its cores into contiguous
    # slices (pinned), and the entropy-coder pool of each rank gets its slice ($MLIC_HOST_THREADS, read
    # at first use)
    cores = sorted(os.sched_getaffinity(0))
    if nloc > 1 and len(cores) >= 2 * nloc:
        k = len(cores) // nloc
        cores = cores[lslot * k:(lslot + 1) * k]
        os.sched_setaffinity(0, cores)
    if "MLIC_HOST_THREADS" not in os.environ:
        os.environ["MLIC_HOST_THREADS"] = str(max(2, min(16, len(cores))))
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from mlic_amd import _lib, bitstream, get_model, synthetic
    from mlic_amd import dist as mdist
    wl = WORKLOADS[a.config]
    jobs, n_jobs_total = build_jobs(a, jrank, jworld)
    groups = batches(jobs, split=a.split)
    # biggest batches first: the concurrent groups finish together
    order = sorted(range(len(groups)), key=lambda gi: -len(groups[gi][1]) * groups[gi][0][2] * groups[gi][0][3])
    conc = max(1, min(a.group_concurrency, len(groups)))
    if a.lanes_auto and len(groups) >= conc and conc > 1:
        # more batches than concurrent slots: the batches overlap each other, one lane each is best
        a.lanes = WORKLOADS[a.config]["lanes_many"]

    # one model instance per group when groups run concurrently (a handle's lanes serve one call at a
    # time), one per weight set otherwise
    nets, gnet = {}, []
    for gi, ((model, rate, _, _), _js) in enumerate(groups):
        key = (model, rate, gi if conc > 1 else 0)
        if key not in nets:
            n = get_model(model)
            n.load_state_dict(synthetic.synth_state_dict(model, 0, rate=rate))
            n = n.to(dev).eval()
            n.update()
            n.set_lanes(a.lanes)
            if conc > 1 and os.environ.get("MLIC_GROUP_PRIO", "0") != "0":
                # A/B (MLIC_GROUP_PRIO=1): staggered stream priorities across the concurrent groups' models
                # (group g's lanes after group g - 1's).  Measured slower (main line 103.8-105.7 vs
                # 105.4-106.5 img/s, profiles/r06/ab/group_priority_ab.log): with 3 priority levels the
                # low-priority groups are starved into a serial tail at the end of every step
                n.set_priority_base(gi * a.lanes)
            n.set_precision(a.precision)
            n.set_synthesis_precision(1 if a.synth_fp16 else 0)
            nets[key] = n
        gnet.append(nets[key])
    # inputs resident in HBM before the timed region
    xs = [torch.cat([synthetic.synth_image(j.H, j.W, j.seed) for j in js]).to(dev) for _, js in groups]
    streams = [torch.cuda.Stream(dev) for _ in groups]
    torch.cuda.synchronize()
    is_vbr = wl["model"].endswith("_VBR")

    split = {"compress": 0.0, "decompress": 0.0}
    last = {}
    decode_only = a.phase == "decode"
    mode = {"decode": decode_only}  # run_group's phase: the decode sub-record flips it after the main region

    def group_kw(gi):
        return {"stage": 2, "s": [j.level for j in groups[gi][1]]} if is_vbr else {}

    # decode phase: every group's streams are encoded once, before the warmup and the timed region
    pre = {}
    if decode_only:
        for gi in range(len(groups)):
            with torch.cuda.stream(streams[gi]):
                pre[gi] = gnet[gi].compress(xs[gi], **group_kw(gi))
        torch.cuda.synchronize()

    def run_group(gi):
        js = groups[gi][1]
        net = gnet[gi]
        kw = group_kw(gi)
        with torch.cuda.stream(streams[gi]):
            t_a = time.perf_counter()
            c = pre[gi] if mode["decode"] else net.compress(xs[gi], **kw)
            t_b = time.perf_counter()
            d = net.decompress(c["strings"], c["shape"], **kw)
            t_c = time.perf_counter()
        last[gi] = (c, d, (t_b - t_a) / len(js), (t_c - t_b) / len(js))
        return t_b - t_a, t_c - t_b

    pool = None
    if conc > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(conc)

    def step():
        res = list(pool.map(run_group, order)) if pool else [run_group(gi) for gi in order]
        for te, td in res:
            split["compress"] += te
            split["decompress"] += td

    # request streams (every batch has its own worker): each runs its n steps back to back, so the
    # streams drift apart instead of meeting at a join every step; the timed region still holds exactly
    # K steps of every batch, bracketed by the same synchronisation
    streams_mode = a.schedule == "streams" and pool is not None and len(order) <= conc

    def run_steps(n):
        if not streams_mode:
            for _ in range(n):
                step()
            return

        def chain(gi):
            return [run_group(gi) for _ in range(n)]
        for res in pool.map(chain, order):
            for te, td in res:
                split["compress"] += te
                split["decompress"] += td

    run_steps(a.warmup)
    torch.cuda.synchronize()
    hs = [C.c_double() for _ in range(3)]
    for n in nets.values():
        _lib.call("mlic_host_stats", n._ensure_handle(dev), *[C.byref(v) for v in hs], 1)
    split["compress"] = split["decompress"] = 0.0
    elapsed = timed_steps(run_steps, a.steps, distributed, dev, sync=torch.cuda.synchronize)
    host = {"rans_encode": 0.0, "rans_decode": 0.0, "gpu_wait": 0.0}
    for n in nets.values():
        _lib.call("mlic_host_stats", n._handle, *[C.byref(v) for v in hs], 1)
        for k, v in zip(host, hs):
            host[k] += v.value / a.steps
    host = {k: round(v, 2) for k, v in host.items()}
    wall_split = {k: round(1000 * v / a.steps, 2) for k, v in split.items()}
    if decode_only:
        wall_split.pop("compress")

    # per-image records (mlic_amd.dist.RECORD_FIELDS): the one collective, all_gather over RCCL/xGMI
    F = {k: i for i, k in enumerate(mdist.RECORD_FIELDS)}
    rec = torch.zeros(len(jobs), mdist.RECORD_LEN, dtype=torch.float64)
    r = 0
    for gi, ((model, rate, H, W), js) in enumerate(groups):
        c, d, enc_s, dec_s = last[gi]
        net = gnet[gi]
        mses = mse_u8(xs[gi], d["x_hat"])
        if gnet.count(net) > 1:
            # the device-side likelihood bits belong to a net's last compress(): groups sharing one
            # net (vbr-mixed's 4K + 1080p) re-run this group's compress, untimed, to read them
            c = net.compress(xs[gi], **group_kw(gi))
        for i, j in enumerate(js):
            # the file the harness writes (header included, utils/utils.py:71-83), as bitstream.write_stream
            nbytes = bitstream.file_bytes(len(c["strings"][0][i]), len(c["strings"][1][i]), vbr=is_vbr)
            yb, zb = net.likelihood_bits(i)
            rec[r, F["job"]] = j.id
            rec[r, F["H"]], rec[r, F["W"]] = H, W
            rec[r, F["level"]] = j.level
            rec[r, F["bytes"]] = nbytes
            rec[r, F["bpp_file"]] = 8.0 * nbytes / (H * W)
            rec[r, F["bpp_lik"]] = (yb + zb) / (H * W)
            rec[r, F["mse"]] = mses[i]
            rec[r, F["psnr"]] = psnr_from_mse(mses[i])
            rec[r, F["enc_ms"]] = 1000 * enc_s
            rec[r, F["dec_ms"]] = 1000 * dec_s
            r += 1
    # every job of the list exactly once (emulated: this rank's share of it)
    allrec = gather_all(rec, len(jobs) if emulated else n_jobs_total, distributed, dev)

    # live roofline: extra profiled (untimed) steps.  Pass 1 runs the timed steps' lane count, so its
    # per-launch averages are what rocprofv3 sees over the whole run (concurrent lanes stretch each
    # launch); pass 2 runs one lane's share of the first batch on one lane (launches of the same
    # shapes, each alone on the GPU).
    roofline = None
    prof = {}
    if not a.no_roofline:
        roofline, prof = profile_roofline(a, gnet, groups, xs, is_vbr, elapsed / a.steps, dev,
                                          pre=pre if decode_only else None)

    # decode sub-record (phase both): north_star states its target for MLICPP_L DECODE, so the default line
    # also times decompress() alone -- K more steps over the streams the timed enc+dec steps produced (the
    # last step's compress() of every request stream), the same request streams and lanes, its own barrier-
    # bracketed region and max over ranks, its own isolated-pass roofline (encoder launches dropped); the
    # decoded x_hat must equal the timed steps' bit for bit
    decode_rec = None
    if not decode_only and not a.no_decode_record:
        enc_last = {gi: last[gi] for gi in range(len(groups))}
        pre.update({gi: enc_last[gi][0] for gi in range(len(groups))})
        mode["decode"] = True
        run_steps(1)  # warmup: the decode-only schedule
        torch.cuda.synchronize()
        elapsed_d = timed_steps(run_steps, a.steps, distributed, dev, sync=torch.cuda.synchronize)
        same = all(torch.equal(last[gi][1]["x_hat"], enc_last[gi][1]["x_hat"]) for gi in range(len(groups)))
        assert same, "decode sub-record: decompress of the timed streams != the timed steps' x_hat"
        rd = None
        if not a.no_roofline:
            rd, _ = profile_roofline(a, gnet, groups, xs, is_vbr, elapsed_d / a.steps, dev, pre=pre,
                                     write_layers=False)
        mode["decode"] = False
        decode_rec = {"elapsed_s": elapsed_d, "roofline": rd, "x_hat_equals_timed_steps": same}

    if rank == 0:
        if emulated:  # this rank's images only: a per-GPU prediction
            images = len(jobs) * a.steps
        else:
            images = n_jobs_total * a.steps if wl["scaling"] == "strong" else len(jobs) * world * a.steps
        q = allrec.numpy()
        quality = {"bpp_file_mean": round(float(q[:, F["bpp_file"]].mean()), 5),
                   "bpp_lik_mean": round(float(q[:, F["bpp_lik"]].mean()), 5),
                   "psnr_u8_mean": round(float(q[:, F["psnr"]].mean()), 4), "images": int(q.shape[0])}
        if a.config in ("kodak-sweep", "vbr-mixed"):
            per = {}
            for lv in sorted(set(int(v) for v in q[:, F["level"]])):
                sel = q[q[:, F["level"]] == lv]
                key = (f"lambda_{synthetic.RATE_LAMBDAS[lv]}" if a.config == "kodak-sweep" else f"vbr_level_{lv}")
                per[key] = {"images": int(sel.shape[0]), "bpp_file": round(float(sel[:, F["bpp_file"]].mean()), 5),
                            "bpp_lik": round(float(sel[:, F["bpp_lik"]].mean()), 5),
                            "psnr": round(float(sel[:, F["psnr"]].mean()), 4)}
            quality["per_level"] = per
        cfg0 = groups[0][0]
        out = {
            "metric": (METRIC if a.config == "main" else f"images/sec (enc+dec), {wl['desc']}") if not decode_only
                      else f"images/sec (decode only: decompress() of streams encoded before the timed region), "
                           f"{wl['desc']}",
            "phase": a.phase,
            "value": round(images / elapsed, 4),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": None,
            "dtype": ("f32" if a.precision == 0 else "f32 (dense convs: f32 via split-fp16 MFMA, 3 terms)")
                     + ("; g_s subpel convs fp16 operands, fp32 accumulate" if a.synth_fp16 else ""),
            "data": "synthetic (seeded sinusoid images; seeded conditioned realistic-rate weights)",
            "config": {"workload": wl["desc"] + " (full rANS bitstreams, inputs resident in HBM)",
                       "name": a.config, "model": wl["model"], "global_batch": n_jobs_total,
                       "per_gpu_images": len(jobs),
                       "shapes": sorted({f"{W}x{H}" for (_, _, H, W), _ in groups}),
                       "weights": ("high-rate set (round 1)" if cfg0[1] is None else
                                   f"rate set(s) {sorted({k[1] for k, _ in groups})} of synthetic.RATE_LAMBDAS"),
                       "parallelism": f"image-sharded x{world} (no cross-GPU context)",
                       "request_streams": len(groups), "lanes_per_stream": a.lanes,
                       "schedule": ("each request stream runs its K steps back to back (no per-step join)"
                                    if streams_mode else "batches joined every step"),
                       **({"synthesis": "fp16 operands (SURVEY f4)"} if a.synth_fp16 else {})},
            "roofline": roofline,
            **prof,
            "host_thread_ms_per_step": host,
            "host_threads": int(os.environ.get("MLIC_HOST_THREADS", "0")),
            # per-phase wall time per step; with concurrent groups the phases of different groups overlap,
            # so the sums may exceed the step (reported under a name that says so)
            ("wall_ms_per_step" if conc == 1 else "wall_ms_per_step_summed_over_concurrent_groups"): wall_split,
            "lanes": a.lanes,
            "group_concurrency": conc,
            "batches_per_step": [len(js) for _, js in groups],
            "quality": quality,
        }
        if decode_rec is not None:
            rd = decode_rec["roofline"]
            out["decode"] = {
                "metric": "images/sec (decode only: decompress() of the timed enc+dec steps' own streams)",
                "value": round(images / decode_rec["elapsed_s"], 4), "unit": "images/sec",
                "ms_per_step": round(1000 * decode_rec["elapsed_s"] / a.steps, 3), "steps": a.steps, "warmup": 1,
                "step_frac": rd["step_frac"] if rd else None,
                "x_hat_equals_timed_steps": decode_rec["x_hat_equals_timed_steps"],
                "roofline": ({k: rd[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac",
                                                  "launches_isolated", "avg_launch_us", "step_t_roof_ms", "step_ms",
                                                  "step_frac", "share_of_isolated_gpu_time")} if rd else None)}
        if emulated:
            out["emulated"] = {"world": a.emulate_world, "rank": a.emulate_rank, "host_cores": len(cores),
                               "note": "one rank's job list of a W-GPU run on one GPU with 1/W of the host cores; "
                                       "value = that rank's images/s (per-GPU)"}
        if world == 1 and not a.no_cpu_baseline:
            # the CPU sample is one of the GPU's own jobs (the first of at most 1080p size): the oracle
            # codes that image, so the headline carries the bpp / PSNR delta against the CPU path on the
            # same input (BASELINE metric "bpp/PSNR delta vs ref"; loss/rd_loss.py:42-45, utils/metrics.py:32-33)
            j0 = next((j for j in jobs if j.H * j.W <= 1088 * 1920), jobs[0])
            out["cpu_baseline"], coded = cpu_baseline(j0.model, j0.rate, min(j0.H, 1088), min(j0.W, 1920),
                                                      j0.level if is_vbr else -1, phase=a.phase, seed=j0.seed)
            if "decode" in out:  # the same oracle run's decoder-side time (decoder network + native rANS decode)
                out["decode"]["cpu_baseline"] = {"value": out["cpu_baseline"]["decode_value"],
                                                 "unit": "images/sec (decode)",
                                                 "cores": out["cpu_baseline"]["cores"], "kind": "port",
                                                 "sample": "the enc+dec cpu_baseline's image, its decoder half"}
            g0 = q[q[:, F["job"]] == j0.id][0]
            if (coded["H"], coded["W"]) == (j0.H, j0.W):
                d_lik = float(g0[F["bpp_lik"]]) - coded["bpp_lik"]
                d_psnr = float(g0[F["psnr"]]) - coded["psnr"]
                out["quality"]["delta_vs_cpu_oracle_job"] = {
                    "job": j0.id, "image": f"{j0.W}x{j0.H} seed {j0.seed}, rate set {j0.rate}"
                                           + (f", VBR level {j0.level}" if is_vbr else ""),
                    "bpp_lik_gpu": round(float(g0[F["bpp_lik"]]), 7), "bpp_lik_cpu": round(coded["bpp_lik"], 7),
                    "d_bpp_lik": round(d_lik, 8),
                    "bpp_file_gpu": round(float(g0[F["bpp_file"]]), 7), "bpp_file_cpu": round(coded["bpp_file"], 7),
                    "d_bpp_file": round(float(g0[F["bpp_file"]]) - coded["bpp_file"], 8),
                    "psnr_gpu": round(float(g0[F["psnr"]]), 6), "psnr_cpu": round(coded["psnr"], 6),
                    "d_psnr_db": round(d_psnr, 7),
                    "within_tolerance": bool(abs(d_lik) <= 1e-3 and abs(d_psnr) <= 1e-2),
                    "tolerance": "north_star: |d bpp| <= 0.001, |d PSNR| <= 0.01 dB (GPU: the timed run's own "
                                 "bitstream and decoded x_hat; CPU: the oracle's encoder, native rANS and decoder)"}
            if a.config == "kodak-sweep":
                out["quality"]["delta_vs_cpu_oracle"] = oracle_deltas(
                    wl["model"], sorted({k[1] for k, _ in groups}), 512, 768,
                    {k[1]: gnet[gi] for gi, (k, _) in enumerate(groups)}, dev)
        else:
            out["cpu_baseline"] = None
        if a.records_out:
            with open(a.records_out, "w") as f:
                json.dump({"fields": list(mdist.RECORD_FIELDS), "records": allrec.tolist()}, f)
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def profile_roofline(a, gnet, groups, xs, is_vbr, t_step_s, dev, pre=None, write_layers=True):
    """pre: the decode phase's pre-encoded streams per group (only decompress launches are counted)."""
    from mlic_amd import _lib
    ncat = C.c_int()
    _lib.call("mlic_profile_categories", C.byref(ncat))
    names = []
    for cat in range(ncat.value):
        nb = C.create_string_buffer(128)
        _lib.call("mlic_profile_category_name", cat, nb, 128)
        names.append(nb.value.decode())

    def profile_pass(lanes, share=None):
        fam = {}
        layer_rows = []
        for gi, ((model, rate, H, W), js) in enumerate(groups):
            net = gnet[gi]
            h = net._handle
            _lib.call("mlic_set_lanes", h, lanes)
            _lib.call("mlic_set_profiling", h, 1)
            x = xs[gi] if share is None else xs[gi][:share]
            kw = {"stage": 2, "s": [j.level for j in js][:x.shape[0]]} if is_vbr else {}

            def harvest(tag):
                n = C.c_size_t()
                _lib.call("mlic_profile_layers", h, None, 0, C.byref(n))
                buf = C.create_string_buffer(n.value + 1)
                _lib.call("mlic_profile_layers", h, buf, n.value + 1, C.byref(n))
                lines = buf.value.decode().splitlines()
                if not layer_rows:
                    layer_rows.append("phase\t" + lines[0])
                layer_rows.extend(f"{tag}\t{ln}" for ln in lines[1:])
                for cat, nm in enumerate(names):
                    n_, ms, fl, by = C.c_int64(), C.c_double(), C.c_double(), C.c_double()
                    _lib.call("mlic_profile_read", h, cat, C.byref(n_), C.byref(ms), C.byref(fl), C.byref(by))
                    if n_.value == 0:
                        continue
                    f = fam.setdefault(family(nm), {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
                    f["launches"] += n_.value
                    f["ms"] += ms.value
                    f["flops"] += fl.value
                    f["bytes"] += by.value

            if pre is None:
                c = net.compress(x, **kw)
                torch.cuda.synchronize()
                harvest("compress")
            else:  # decode phase: the streams of the timed steps (the isolated pass: its first images')
                c = pre[gi] if share is None else net.compress(x, **kw)
                torch.cuda.synchronize()
                for cat in range(ncat.value):  # drop the encoder's launches
                    _lib.call("mlic_profile_read", h, cat, *[C.byref(v) for v in (C.c_int64(), C.c_double(),
                                                                                  C.c_double(), C.c_double())])
            net.decompress(c["strings"], c["shape"], **kw)
            torch.cuda.synchronize()
            harvest("decompress")
            _lib.call("mlic_set_profiling", h, 0)
            _lib.call("mlic_set_lanes", h, a.lanes)
            if share is not None:
                break  # the isolated pass profiles one lane's share of the first batch only
        return fam, layer_rows

    prof_lanes = a.profile_lanes or a.lanes
    fam, _ = profile_pass(prof_lanes)
    # isolated pass: one lane on 8 images of the first batch (the r04 records' unit: bench.py --lanes 1
    # --batch 8 --split 1 under rocprofv3 profiles the same launches)
    share = min(8, len(groups[0][1]))
    fam1, layer_rows1 = profile_pass(1, share)
    if write_layers and a.layers_out and int(os.environ.get("RANK", "0")) == 0:
        with open(a.layers_out, "w") as f:  # isolated launches: the per-layer efficiency table
            f.write("\n".join(layer_rows1) + "\n")

    def bound_of(fm, name):
        peak_tf, arith = kernel_peak(name)
        ai = fm["flops"] / max(fm["bytes"], 1.0)
        if fm["flops"] <= 0 or ai * PEAK_HBM_GBS * 1e9 < peak_tf * 1e12:
            return "hbm", "GB/s", fm["bytes"] / (max(fm["ms"], 1e-9) * 1e-3) / 1e9, PEAK_HBM_GBS, arith
        return "mfma", "TFLOP/s", fm["flops"] / (max(fm["ms"], 1e-9) * 1e-3) / 1e12, peak_tf, arith

    def t_roof_ms(fm, name):
        peak_tf, _ = kernel_peak(name)
        return 1e3 * max(fm["flops"] / (peak_tf * 1e12), fm["bytes"] / (PEAK_HBM_GBS * 1e9))

    # The headline roofline is the kernel's own: launch durations of the isolated pass (one lane running
    # one lane's share of the first batch, each launch alone on the GPU -- reproducible with
    # `rocprofv3 --kernel-trace --stats -- python bench.py --lanes 1 --batch 8 --split 1`).  The timed
    # configuration's launches overlap across lanes, so their HIP-event durations include other lanes'
    # kernels; they are kept as the secondary `concurrent` entry.
    # dominant = the family with the most isolated device time
    dom = max(fam1, key=lambda k: fam1[k]["ms"]) if fam1 else max(fam, key=lambda k: fam[k]["ms"])
    iso = fam1.get(dom) or fam[dom]
    bound, unit, achieved, peak, arith = bound_of(iso, dom)
    t_roof = sum(t_roof_ms(v, k) for k, v in fam.items())
    traffic, traffic_src = None, None
    try:
        with open(a.traffic_json) as f:
            tj = json.load(f)
        if tj.get("config", "main") == a.config and family(tj.get("family", "")) == dom:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = tj.get("launches_of")
    except (OSError, ValueError):
        pass
    # the isolated pass covers `share` images of the first batch; scaled to the step's pixels, the
    # family's own time per step cannot exceed the measured step (it is one family of many)
    step_px = sum(len(js) * H * W for (_, _, H, W), js in groups)
    share_px = share * groups[0][0][2] * groups[0][0][3]
    dom_ms_step = iso["ms"] * step_px / share_px
    assert dom_ms_step <= 1e3 * t_step_s, (dom, dom_ms_step, 1e3 * t_step_s)
    roofline = {"bound": bound, "kernel": f"{dom} ({arith})",
                "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": unit,
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_launches": traffic_src,
                "timing": f"isolated: HIP events around each launch, one lane, {share} image(s) of the first "
                          f"batch, each launch alone on the GPU",
                "launches_isolated": iso["launches"], "avg_launch_us": round(1000 * iso["ms"] / max(1, iso["launches"]), 2),
                "algorithmic_flops_per_launch": round(iso["flops"] / max(1, iso["launches"])),
                "algorithmic_bytes_per_launch": round(iso["bytes"] / max(1, iso["launches"])),
                "family_ms_per_step_from_isolated": round(dom_ms_step, 3),
                "share_of_isolated_gpu_time": round(iso["ms"] / max(1e-9, sum(v["ms"] for v in fam1.values())), 4),
                # T_roof = sum_k max(F_k / P_k, B_k / BW) over every kernel of one step,
                # against the measured step time
                "step_t_roof_ms": round(t_roof, 3), "step_ms": round(1e3 * t_step_s, 3),
                "step_frac": round(t_roof / max(1e-9, 1e3 * t_step_s), 4)}
    if dom in fam:
        _, _, ach_c, _, _ = bound_of(fam[dom], dom)
        roofline["concurrent"] = {"achieved": round(ach_c, 3), "frac": round(ach_c / peak, 4),
                                  "lanes": prof_lanes, "launches_per_step": fam[dom]["launches"],
                                  "avg_launch_us": round(1000 * fam[dom]["ms"] / max(1, fam[dom]["launches"]), 2),
                                  "note": "launches of the timed configuration, overlapped across lanes"}
    # the runner-up families (isolated), each with its own roofline fraction
    others = []
    for k in sorted(fam1, key=lambda k: -fam1[k]["ms"])[1:4]:
        b_, u_, a_, p_, _ = bound_of(fam1[k], k)
        others.append({"kernel": k, "bound": b_, "achieved": round(a_, 3), "peak": round(p_, 1), "unit": u_,
                       "frac": round(a_ / p_, 4), "launches_isolated": fam1[k]["launches"],
                       "avg_launch_us": round(1000 * fam1[k]["ms"] / max(1, fam1[k]["launches"]), 2),
                       "share_of_isolated_gpu_time": round(fam1[k]["ms"] / max(1e-9, sum(v["ms"] for v in fam1.values())), 4)})
    roofline["runners_up"] = others
    prof = {
        # with profile_lanes > 1 these are per-launch durations summed over concurrently running lanes
        "kernel_families_ms_per_step": {k: round(v["ms"], 3) for k, v in sorted(fam.items(), key=lambda kv: -kv[1]["ms"])},
        "gpu_kernel_ms_per_step": round(sum(v["ms"] for v in fam.values()), 3),
        "kernel_families_ms_isolated_share": {k: round(v["ms"], 3)
                                              for k, v in sorted(fam1.items(), key=lambda kv: -kv[1]["ms"])},
        "gpu_kernel_ms_isolated_share": round(sum(v["ms"] for v in fam1.values()), 3),
        "isolated_share_images": share,
        "profile_lanes": prof_lanes,
    }
    return roofline, prof


if __name__ == "__main__":
    main()
