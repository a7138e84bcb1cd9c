"""Benchmark of the MI355X OpenPose path: frames/s end-to-end (CNN + PAF grouping) at 368x368.

python bench.py [--gpus N --steps K --warmup W --batch B]
For N > 1 launch with torch.distributed.run (one process per GPU, RCCL gather of the per-frame
result records to every rank).  A step = one batch of B frames per GPU through the whole path:
uint8 BGR frame in HBM -> resize + normalise -> 92 convs -> upsample / Gaussian / NMS ->
line integrals -> greedy assignment -> grouping -> poses copied to the host.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for every field.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "chainer_realtime_multi-person_pose_estimation_amd"
METRIC = "frames/sec end-to-end (CNN+PAF grouping) at 368×368, 1/2/4/8 MI355X"
FP32_MATRIX_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense MFMA peak
HBM_PEAK_GBS = 8000.0
PARAMS_SCALES = [0.5, 1, 1.5, 2]  # entity.py:74 inference_scales


def precise_net(h, w, scale, size=368, stride=8):
    """detect_precise's padded network input for one scale (pose_detector.py:440-447): (net_h, net_w)."""
    import math
    m = scale * size / min(h, w)
    rh, rw = math.ceil(h * m), math.ceil(w * m)
    return rh + (-rh) % stride, rw + (-rw) % stride


def synthetic_maps(batch, lh=46, lw=46):
    """COCO-like last-stage maps (38 PAF + 19 heat) from the reference's own label generators
    (tests/golden/*.npz, made by tests/golden/make_golden.py): 6 people at 46x46 (368x368 frames),
    20 people at 46x82 (1280x720 frames); None for other map sizes."""
    name = {(46, 46): "six_people", (46, 82): "twenty_720p"}.get((lh, lw))
    if name is None:
        return None
    d = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
    m = np.concatenate([d["paf_low"], d["heat_low"]])[None]
    return np.ascontiguousarray(np.repeat(m, batch, axis=0))


def optimal_size(h, w, size=368, stride=8):
    """compute_optimal_size (pose_detector.py:57-73): (net_w, net_h)."""
    if w < h:
        ow = size
        oh = np.round(size * h / w)
    else:
        oh = size
        ow = np.round(size * w / h)
    ow, oh = int(ow), int(oh)
    return ow + (-ow) % stride, oh + (-oh) % stride


def cpu_baseline(frames, maps, n_frames):
    """The oracle (NumPy Chainer-CPU forward + C post-process restatement), timed per frame."""
    from oracle import forward as F
    from oracle import cvresize, postproc as P
    import importlib
    W = importlib.import_module(PKG + ".weights").random_weights(seed=0)
    try:
        from threadpoolctl import threadpool_info
        cores = max([int(i.get("num_threads", 1)) for i in threadpool_info()] + [1])
    except Exception:
        cores = os.cpu_count() or 1
    x = cvresize.preprocess(cvresize.resize_linear_u8(frames[0], 368, 368))
    F.cocoposenet_forward(W, x)  # warm-up
    t0 = time.perf_counter()
    for i in range(n_frames):
        f = frames[i % len(frames)]
        x = cvresize.preprocess(cvresize.resize_linear_u8(f, 368, 368))
        F.cocoposenet_forward(W, x)
        P.postprocess(maps[i % len(maps), :38], maps[i % len(maps), 38:], f.shape[0], f.shape[1])
    dt = time.perf_counter() - t0
    return {"value": n_frames / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": "%d frames: oracle im2col+sgemm forward (368x368, NumPy BLAS) + C post-process "
                      "restatement on the same 6-person maps; %.1f s total" % (n_frames, dt)}


KERNEL_7X7 = {0: "conv_bf16x3<7", 1: "conv7_halo_bf16x3", 2: "conv7_halo_bf16x3", 3: "conv_halo_bf16x3<7",
              4: "conv_m16_bf16x3<7", 5: "conv_m16_bf16x3<7", 6: "conv_pair_bf16x3<7", 7: "conv_db_bf16x3<7",
              8: "conv_m16_bf16x3<7", 9: "conv_big_bf16x3<7", 10: "conv_big_bf16x3<7", 11: "conv_big_bf16x3<7"}
MFMA_7X7 = {4: "v_mfma_f32_16x16x32_bf16", 5: "v_mfma_f32_16x16x32_bf16", 6: "v_mfma_f32_16x16x32_bf16",
            8: "v_mfma_f32_16x16x32_bf16"}


def committed_traffic(kernel, batch, precision, halo_mode):
    """HBM bytes per launch (read + write) of `kernel` from the newest committed rocprofv3 PMC
    summary (profiles/*_traffic.json, FETCH_SIZE x calibrated pattern factor + WRITE_SIZE, tools/summarize_profile.py) taken
    on this exact workload; (None, None) when no profile matches."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        cfg = d.get("config") or {}
        if cfg.get("frames_per_step_per_gpu") != batch or d.get("precision", "bf16x3") != precision:
            continue
        if KERNEL_7X7.get(d.get("halo_mode", 1)) != KERNEL_7X7.get(halo_mode):  # same 7x7 kernel
            continue
        for k, v in d.get("kernels", {}).items():
            if k.replace("op::", "").startswith(kernel):
                best = (int(v["read_bytes"] + v["write_bytes"]), os.path.basename(p))
    return best if best else (None, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=38,
                    help="frames per step per GPU (38: the 7x7 kernel's 640-pixel raster tiles, "
                         "ceil(38 x 2116 / 640) = 126 per branch x 2 = 252 workgroups, one per CU)")
    ap.add_argument("--maps", choices=["synthetic", "network"], default="synthetic",
                    help="post-process input: COCO-like 6-person maps (default) or the random-weight "
                         "network's own last stage")
    ap.add_argument("--cpu-frames", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--graph", type=int, default=0, help="1: replay each step as one captured hipGraph")
    ap.add_argument("--precision", choices=["bf16x3", "fp32"], default="bf16x3",
                    help="conv arithmetic: 3xBF16-split products (f32 accumulate) or exact f32 MFMA")
    ap.add_argument("--frame", default="368x368",
                    help="HxW of the synthetic frames (BASELINE configs: 368x368 = C2/C3, the default "
                         "and the headline; 720x1280 = C5's 720p stream, single scale)")
    ap.add_argument("--precise", action="store_true",
                    help="C4: multi-scale detect_precise (4 scales, cubic resizes) on the staged batch "
                         "(op_run_staged_precise: one batched forward per scale)")
    args = ap.parse_args()
    FH, FW = (int(v) for v in args.frame.lower().split("x"))
    headline = (FH, FW) == (368, 368) and not args.precise
    if not headline:
        args.no_cpu_baseline = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # OP_BENCH_BACKEND=gloo (rehearsal only: N ranks sharing the GPUs of a smaller box, CPU-side
    # collectives); the product path is RCCL ('nccl'), one rank per GPU
    backend = os.environ.get("OP_BENCH_BACKEND", "nccl")
    coll_dev = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            coll_dev = torch.device("cuda", local)
        else:
            local = local % max(1, torch.cuda.device_count())
            dist.init_process_group(backend)
    import importlib
    L = importlib.import_module(PKG + "._lib")
    Wm = importlib.import_module(PKG + ".weights")
    Fr = importlib.import_module(PKG + ".frames")

    B = args.batch
    net_w, net_h = optimal_size(FH, FW)
    halo_mode = int(os.environ.get("OP_HALO_MODE", "4"))
    limits = L.OpLimits()
    limits.max_batch = B
    ctx = L.Context(local, None, limits)
    ctx.set_precision(args.precision)
    wts = Wm.random_weights(seed=0)
    if args.precise:
        # the random network's 1280x720 maps are noise with thousands of spurious peaks per joint
        # (past the per-frame caps); a -1 bias on the last stage's Mconv7 keeps them below the peak
        # threshold -- same FLOPs, the post-process still runs its full-resolution passes
        for k in ("Mconv7_stage6_L1", "Mconv7_stage6_L2"):
            wts[k] = (wts[k][0], wts[k][1] - np.float32(1.0))
    ctx.set_weights(wts)
    rng = np.random.default_rng(1234 + rank)
    frames = rng.integers(0, 256, (B, FH, FW, 3), dtype=np.uint8)
    maps = synthetic_maps(B, net_h // 8, net_w // 8)
    if maps is None or args.precise:
        args.maps = "network"
    ctx.stage_frames(frames)
    if not args.precise:
        if args.maps == "synthetic":
            ctx.stage_maps(maps)
            ctx.use_staged_maps(True)

    def barrier():
        if dist is not None:
            import torch
            dist.all_reduce(torch.zeros(1, device=coll_dev))
            if coll_dev is not None:
                torch.cuda.synchronize()

    persons = 0

    def step(collect):
        nonlocal persons
        if args.precise:
            ctx.run_staged_precise()
            res = ctx.fetch_results(0, B)
        else:
            ctx.run_staged(graph=bool(args.graph))
            ctx.synchronize()
            res = ctx.fetch_results(0, B)
        if collect:
            persons += sum(r[2].n_persons for r in res)
        if dist is not None:
            import torch
            recs = Fr.pack_records([(rank + world * i, r[2].status, r[2].n_peaks, r[0], r[1])
                                    for i, r in enumerate(res)], 64)
            Fr.gather_records(recs, 64, device=coll_dev)

    for _ in range(args.warmup):
        step(False)
    ctx.synchronize()
    # timed region: HIP events only around the dominant kernel (the 7x7 stage convs) for the
    # roofline, so the per-launch event overhead stays off the other ~90 launches of a step
    ctx.profile_classes(["conv7x7"])
    ctx.profile(not args.no_profile and not args.graph)
    ctx.profile_reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    ctx.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    # per-class breakdown from a few extra (untimed) steps with every class evented
    ctx.profile_classes(list(ctx.PROFILE_CLASSES))
    ctx.profile(not args.no_profile)
    ctx.profile_reset()
    n_extra = 0 if args.no_profile else 3
    for _ in range(n_extra):
        if args.precise:
            step(False)
        else:
            ctx.run_staged()
            ctx.synchronize()
    prof_all = ctx.profile_read()
    ctx.profile(False)
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        pt = torch.tensor([float(persons)], device=coll_dev, dtype=torch.float64)
        dist.all_reduce(pt)
        persons = float(pt.item())

    frames_total = world * B * args.steps
    value = frames_total / elapsed
    ms7, n7, fl7, by7 = prof["conv7x7"]
    roofline = None
    if n7 > 0 and ms7 > 0:
        achieved = fl7 / (ms7 * 1e-3) / 1e12
        if args.precision == "bf16x3":
            # 3 bf16 MFMA products per f32-accurate MAC: the f32-accurate peak is 2500/3 TFLOP/s
            peak = BF16_DENSE_PEAK_TFLOPS / 3.0
            kern = "%s (7x7 stage convs, 3xBF16 split on %s)" % (
                KERNEL_7X7.get(halo_mode, "conv_bf16x3<7"), MFMA_7X7.get(halo_mode, "v_mfma_f32_32x32x16_bf16"))
        else:
            peak = FP32_MATRIX_PEAK_TFLOPS
            kern = "conv_mfma_f32<7,2,2> (7x7 stage convs, v_mfma_f32_32x32x2_f32)"
        traffic, tsrc = committed_traffic(kern.split(" ")[0], B, args.precision, halo_mode)
        roofline = {"bound": "mfma", "kernel": kern,
                    "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": tsrc,
                    "launch_ms": round(ms7 / n7, 4), "flops_per_launch": fl7 / n7,
                    "algorithmic_bytes_per_launch": by7 / n7}
    stage_ms = {k: round(v[0] / n_extra, 3) for k, v in prof_all.items()} if n_extra else {}
    metric = METRIC if headline else "frames/sec end-to-end (CNN+PAF grouping) at %dx%d%s, 1/2/4/8 MI355X" % (
        FW, FH, " multi-scale (%s)" % "/".join(str(v) for v in PARAMS_SCALES) if args.precise else "")
    out = {
        "metric": metric, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16x3 (hi/lo split operands, f32 accumulate)" if args.precision == "bf16x3" else "f32",
        "data": "synthetic: seeded uint8 %dx%d BGR frames %s; random-init CocoPoseNet (He-normal); " % (
            FW, FH, "resident in HBM (last-stage biases -1: no spurious peaks on the random network's "
                    "full-resolution maps)" if args.precise else "resident in HBM")
                + ("post-process fed COCO-like %s network maps (reference label generators)"
                   % ("6-person" if (FH, FW) == (368, 368) else "20-person") if args.maps == "synthetic"
                   else "post-process fed the network's own last stage"),
        "config": {"workload": "%dx%d frames, full PoseDetector.%s path (resize+normalise, 92-conv "
                               "CocoPoseNet fp32, PAF post-process), batch of %d frames per GPU per step"
                               % (FW, FH, "detect_precise" if args.precise else "__call__", B),
                   "frames_per_step_per_gpu": B, "net_input": "%dx%d" % (net_w, net_h),
                   "heatmap": "%dx%d" % optimal_size(FH, FW, 320) if not args.precise else "%dx%d" % (FW, FH),
                   "maps": args.maps, "parallelism": "frame-parallel replicas x%d (RCCL gather of results)" % world},
        "persons_per_s": round(persons / elapsed, 2),
        "gflop_per_frame": round((sum(L.forward_flops(*precise_net(FH, FW, sc)) for sc in PARAMS_SCALES)
                                  if args.precise else L.forward_flops(net_h, net_w)) / 1e9, 2),
        "stage_ms_per_step": stage_ms,
        "stage_ms_note": "HIP-event sums per kernel class over %d untimed profiled steps" % n_extra,
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(frames, maps, args.cpu_frames)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
