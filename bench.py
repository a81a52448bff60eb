"""MLIC++ encode+decode throughput on MI355X (BASELINE.json config 2).

One step = compress() + decompress() of a batch of synthetic 1920x1088 images on each GPU with
MLICPP_L (seeded conditioned weights; no checkpoints offline).  Images shard across ranks (one
process per GPU, weak scaling); the only collective is an all_gather of fixed-size per-image
records (bpp/PSNR/bytes) after the timed region — SURVEY §8(e).

    python bench.py [--gpus N --steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  `roofline` is the dominant kernel family (the MFMA implicit-GEMM
conv, ~95 % of the FLOPs) measured live with HIP events on the executor's stream in an extra,
untimed step; `cpu_baseline` times the CPU oracle (torch fp32, this box's cores) on one image.
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

# dense peak of the arithmetic each kernel family runs on (MI355X_MICROARCH.md): fp32 MFMA 157.3 TF;
# the split-fp16 kernels issue 3 fp16 MFMAs (2.5 PF dense) per fp32 product => 2500/3 TF of
# fp32-equivalent work; the VALU conv kernels run exact fp32 FMAs (157.3 TF with packed FMA)
def kernel_peak(name: str):
    if name.startswith(("conv_f16x3", "conv_x3v2", "pw_resident", "conv_halo")):
        return 2500.0 / 3, "3 x v_mfma_f32_32x32x16_f16 per fp32 product (split-fp16)"
    if name.startswith("conv_x4"):
        return 2500.0 / 3, "3 x v_mfma_f32_16x16x32_f16 per fp32 product (split-fp16, LDS-DMA staged)"
    if name.startswith("conv_mfma"):
        return 157.3, "v_mfma_f32_32x32x2_f32"
    return 157.3, "fp32 VALU FMA"


def is_conv(name: str) -> bool:
    return name.startswith(("conv", "pw_resident"))


METRIC = "images/sec (enc+dec) at 1920×1088 MLICPP_L, 1/2/4/8 GPU; bpp/PSNR Δ vs ref"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix peak (dense, exact f32)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU per step")
    ap.add_argument("--model", default="MLICPP_L")
    ap.add_argument("--height", type=int, default=1088)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--lanes", type=int, default=int(os.environ.get("MLIC_LANES", "4")),
                    help="host threads x HIP streams per GPU for compress/decompress")
    ap.add_argument("--precision", type=int, default=int(os.environ.get("MLIC_PRECISION", "2")),
                    help="dense-conv arithmetic: 2 = split-fp16 MFMA v2 + specialised kernels, "
                         "1 = f16x3 v1 tiles, 0 = fp32 MFMA")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--layers-out", default="", help="write the per-layer conv timing table here")
    ap.add_argument("--profile-lanes", type=int, default=0,
                    help="lanes of the profiled step (0 = same as --lanes, so its launches match the timed "
                         "steps' and rocprofv3's per-kernel averages; 1 = isolated per-kernel times)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"),
                    help="PMC-derived HBM bytes per conv launch (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def psnr_u8(a: torch.Tensor, b: torch.Tensor) -> float:
    """utils/utils.py:86-87 (clamp, *255, truncate) + utils/metrics.py:32-33."""
    qa = (a.clamp(0, 1) * 255).to(torch.uint8).float()
    qb = (b.clamp(0, 1) * 255).to(torch.uint8).float()
    mse = torch.mean((qa - qb) ** 2).item()
    return 20 * math.log10(255.0) - 10 * math.log10(mse) if mse > 0 else float("inf")


def cpu_baseline(model: str, H: int, W: int):
    """Oracle (torch CPU fp32 restatement of the reference) enc+dec of one image, with the native
    rANS coder for the entropy-coding part; threads = this process's CPU affinity (<= 32)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mlic_ref_cpu as ref
    from mlic_amd import entropy, synthetic
    cores = max(1, min(32, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    sd = synthetic.synth_state_dict(model, 0)
    m = ref.RefMLIC(model, sd)
    x = synthetic.synth_image(H, W, 0)
    tables = entropy.gaussian_tables(entropy.get_scale_table())
    t0 = time.time()
    st = m.compress_streams(x)
    sym = torch.cat([p[0].reshape(-1) for p in st["phases"]]).numpy()
    idx = torch.cat([p[1].reshape(-1) for p in st["phases"]]).numpy()
    data = entropy.rans_encode(sym, idx, *tables[:3])
    dec = entropy.rans_decode(data, idx, *tables[:3])
    # decoder network: phases fed from the decoded symbols
    offs = np.cumsum([0] + [p[0].numel() for p in st["phases"]])
    phase_syms = [torch.from_numpy(dec[offs[k]:offs[k + 1]]).reshape(st["phases"][k][0].shape)
                  for k in range(len(st["phases"]))]
    m.decode_streams(st["z_symbols"], phase_syms)
    dt = time.time() - t0
    return {"value": round(1.0 / dt, 5), "unit": "images/sec (enc+dec)", "cores": cores, "kind": "port",
            "sample": f"1 image {W}x{H} {model}: oracle torch-CPU fp32 encoder+decoder networks + native rANS, "
                      f"{dt:.1f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from mlic_amd import _lib, get_model, synthetic
    from mlic_amd import dist as mdist
    net = get_model(a.model)
    net.load_state_dict(synthetic.synth_state_dict(a.model, 0))
    net = net.to(dev).eval()
    net.update()
    net.set_lanes(a.lanes)
    net.set_precision(a.precision)
    B, H, W = a.batch, a.height, a.width
    x = torch.cat([synthetic.synth_image(H, W, 1000 * rank + i) for i in range(B)]).to(dev)

    split = {"compress": 0.0, "decompress": 0.0}

    def step():
        t_a = time.perf_counter()
        c = net.compress(x)
        torch.cuda.synchronize()
        t_b = time.perf_counter()
        d = net.decompress(c["strings"], c["shape"])
        torch.cuda.synchronize()
        split["compress"] += t_b - t_a
        split["decompress"] += time.perf_counter() - t_b
        return c, d

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    hs = [C.c_double() for _ in range(3)]
    _lib.call("mlic_host_stats", net._ensure_handle(dev), *[C.byref(v) for v in hs], 1)
    split["compress"] = split["decompress"] = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        c, d = step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _lib.call("mlic_host_stats", net._handle, *[C.byref(v) for v in hs], 1)
    host = {k: round(v.value / a.steps, 2) for k, v in zip(("rans_encode", "rans_decode", "gpu_wait"), hs)}
    wall_split = {k: round(1000 * v / a.steps, 2) for k, v in split.items()}
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # per-image records: the one collective (all_gather over RCCL/xGMI), mlic_amd.dist
    F = {k: i for i, k in enumerate(mdist.RECORD_FIELDS)}
    rec = torch.zeros(B, mdist.RECORD_LEN, dtype=torch.float64)
    for i in range(B):
        nbytes = len(c["strings"][0][i]) + len(c["strings"][1][i])
        rec[i, F["job"]] = rank * B + i
        rec[i, F["H"]], rec[i, F["W"]] = H, W
        rec[i, F["bytes"]] = nbytes
        rec[i, F["bpp_file"]] = 8.0 * nbytes / (H * W)
        rec[i, F["psnr"]] = psnr_u8(x[i], d["x_hat"][i])
    rec = mdist.gather_records(rec.to(dev), max_per_rank=B).cpu()
    rec = rec[:, [F["bytes"], F["bpp_file"], F["psnr"]]]

    # live roofline of the dominant kernel family: extra profiled (untimed) steps.  Pass 1 runs the
    # timed steps' lane count, so its per-launch averages are what rocprofv3 sees over the whole run
    # (concurrent lanes stretch each launch); pass 2 runs one lane's share of the batch on one lane:
    # launches of exactly the same shapes, each alone on the GPU.
    h = net._handle
    ncat = C.c_int()
    _lib.call("mlic_profile_categories", C.byref(ncat))
    names = []
    for cat in range(ncat.value):
        nb = C.create_string_buffer(128)
        _lib.call("mlic_profile_category_name", cat, nb, 128)
        names.append(nb.value.decode())

    def profile_pass(lanes, xs):
        _lib.call("mlic_set_lanes", h, lanes)
        _lib.call("mlic_set_profiling", h, 1)
        fam = {nm: {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0} for nm in names}
        layer_rows, phase_gpu = [], {}

        def harvest(tag):
            # per-layer table (before the reads, which clear), then per-family sums
            n = C.c_size_t()
            _lib.call("mlic_profile_layers", h, None, 0, C.byref(n))
            buf = C.create_string_buffer(n.value + 1)
            _lib.call("mlic_profile_layers", h, buf, n.value + 1, C.byref(n))
            lines = buf.value.decode().splitlines()
            if not layer_rows:
                layer_rows.append("phase\t" + lines[0])
            layer_rows.extend(f"{tag}\t{ln}" for ln in lines[1:])
            tot = 0.0
            for cat, nm in enumerate(names):
                n, ms, fl, by = C.c_int64(), C.c_double(), C.c_double(), C.c_double()
                _lib.call("mlic_profile_read", h, cat, C.byref(n), C.byref(ms), C.byref(fl), C.byref(by))
                f = fam[nm]
                f["launches"] += n.value
                f["ms"] += ms.value
                f["flops"] += fl.value
                f["bytes"] += by.value
                tot += ms.value
            phase_gpu[tag] = round(tot, 3)

        c = net.compress(xs)
        torch.cuda.synchronize()
        harvest("compress")
        net.decompress(c["strings"], c["shape"])
        torch.cuda.synchronize()
        harvest("decompress")
        _lib.call("mlic_set_profiling", h, 0)
        return fam, phase_gpu, layer_rows

    prof_lanes = a.profile_lanes or a.lanes
    fam, phase_gpu, layer_rows = profile_pass(prof_lanes, x)
    share = max(1, B // prof_lanes)
    fam1, phase_gpu1, layer_rows1 = (profile_pass(1, x[:share]) if prof_lanes != 1
                                     else (fam, phase_gpu, layer_rows))
    net.set_lanes(a.lanes)
    if a.layers_out and rank == 0:
        with open(a.layers_out, "w") as f:  # isolated launches: the per-layer efficiency table
            f.write("\n".join(layer_rows1) + "\n")

    def roof(fam, dom):
        conv = fam[dom]
        peak_tf, arith = kernel_peak(dom)
        sec = max(conv["ms"], 1e-9) * 1e-3
        ai = conv["flops"] / max(conv["bytes"], 1.0)
        if ai * PEAK_HBM_GBS * 1e9 < peak_tf * 1e12:
            return "hbm", "GB/s", conv["bytes"] / sec / 1e9, PEAK_HBM_GBS, arith, conv
        return "mfma", "TFLOP/s", conv["flops"] / sec / 1e12, peak_tf, arith, conv

    # dominant kernel = the conv kernel family with the most device time when every launch runs alone
    # (the isolated pass: a property of the kernels, not of how the lanes happened to interleave); its
    # roofline bound is whichever ceiling is lower at its arithmetic intensity (algorithmic FLOPs / bytes)
    convs = [k for k in fam if is_conv(k)]
    dom = max(convs, key=lambda k: fam1[k]["ms"])
    bound, unit, achieved, peak, arith, conv = roof(fam, dom)
    _, _, achieved1, _, _, conv1 = roof(fam1, dom)
    conv_all = {k: sum(fam[c][k] for c in convs) for k in ("launches", "ms", "flops")}
    traffic = None
    try:
        with open(a.traffic_json) as f:
            tj = json.load(f)
        if (tj.get("model") == a.model and tj.get("H") == H and tj.get("W") == W
                and tj.get("family", "") and tj["family"].replace(" ", "") in dom.replace(" ", "")):
            traffic = tj.get("conv_hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    step_gpu_ms = sum(v["ms"] for v in fam.values())

    if rank == 0:
        images = B * world * a.steps
        out = {
            "metric": METRIC,
            "value": round(images / elapsed, 4),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if a.precision == 0 else "f32 (dense convs: f32 via split-fp16 MFMA, 3 terms)",
            "data": "synthetic (seeded sinusoid images, seeded conditioned weights)",
            "config": {"workload": f"{a.model} compress+decompress (full rANS bitstreams) of {W}x{H} images",
                       "model": a.model, "global_batch": B * world, "per_gpu_batch": B, "H": H, "W": W,
                       "parallelism": f"image-sharded x{world} (no cross-GPU context)"},
            "roofline": {"bound": bound, "kernel": f"{dom} ({arith})",
                         "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": unit,
                         "frac": round(achieved / peak, 4),
                         "traffic": traffic,
                         "launches_per_step": conv["launches"],
                         "avg_launch_us": round(1000 * conv["ms"] / max(1, conv["launches"]), 2),
                         "algorithmic_flops_per_launch": round(conv["flops"] / max(1, conv["launches"])),
                         "algorithmic_bytes_per_launch": round(conv["bytes"] / max(1, conv["launches"])),
                         "all_conv_tflops": round(conv_all["flops"] / max(1e-9, conv_all["ms"] * 1e-3) / 1e12, 3),
                         # the same kernel family, same launch shapes, every launch alone on the GPU
                         # (one lane running one lane's share of the batch)
                         "isolated": {"achieved": round(achieved1, 3), "frac": round(achieved1 / peak, 4),
                                      "images": share,
                                      "launches_per_step": conv1["launches"],
                                      "avg_launch_us": round(1000 * conv1["ms"] / max(1, conv1["launches"]), 2)}},
            # with profile_lanes > 1 these are per-launch durations summed over concurrently running lanes
            "kernel_families_ms_per_step": {k: round(v["ms"], 3) for k, v in fam.items() if v["launches"]},
            "gpu_kernel_ms_per_step": round(step_gpu_ms, 3),
            "gpu_kernel_ms_by_phase": phase_gpu,
            # one lane's share of the batch, every launch alone on the GPU (x lanes = one step's work)
            "kernel_families_ms_isolated_share": {k: round(v["ms"], 3) for k, v in fam1.items() if v["launches"]},
            "gpu_kernel_ms_isolated_share": round(sum(v["ms"] for v in fam1.values()), 3),
            "isolated_share_images": share,
            "profile_lanes": prof_lanes,
            "host_thread_ms_per_step": host,
            "wall_ms_per_step": wall_split,
            "lanes": a.lanes,
            "quality": {"bpp_file_mean": round(float(rec[:, 1].mean()), 5),
                        "psnr_u8_mean": round(float(rec[:, 2].mean()), 4), "images": int(rec.shape[0])},
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.model, H, W)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
