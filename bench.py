"""Benchmark of the MI355X OpenPose path: frames/s end-to-end (CNN + PAF grouping) at 368x368.

python bench.py [--gpus N --steps K --warmup W --batch B]
For N > 1 launch one process per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT; nothing here imports PyTorch): frames shard round-robin over the ranks,
and each step's per-frame result records are gathered to rank 0 by RCCL from device memory
(frames.RcclGather / gather.hip), overlapped with the next step.

A step = one batch of B frames per GPU through the whole PoseDetector.__call__ path:
  pinned host frames --(copy stream, overlapped with the previous step)--> HBM ring ->
  resize + normalise -> 92 convs -> upsample / Gaussian / NMS -> line integrals -> greedy
  assignment -> grouping -> poses copied to the host (and, N > 1, gathered to rank 0).

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for every field.
"""
import argparse
import json
import os
import re
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "chainer_realtime_multi-person_pose_estimation_amd"
METRIC = "frames/sec end-to-end (CNN+PAF grouping) at 368×368, 1/2/4/8 MI355X"
FP32_MATRIX_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense MFMA peak
PARAMS_SCALES = [0.5, 1, 1.5, 2]  # entity.py:72 inference_scales
GATHER_PERSONS = 64  # persons carried per frame record (~28 KB per frame)


def precise_net(h, w, scale, size=368, stride=8):
    """detect_precise's padded network input for one scale (pose_detector.py:440-447): (net_h, net_w)."""
    import math
    m = scale * size / min(h, w)
    rh, rw = math.ceil(h * m), math.ceil(w * m)
    return rh + (-rh) % stride, rw + (-rw) % stride


def golden_maps(lh, lw):
    """COCO-like last-stage maps (38 PAF + 19 heat) from the reference's own label generators
    (tests/golden/*.npz, made by tests/golden/make_golden.py): 6 people at 46x46 (368x368 frames),
    20 people at 46x82 (1280x720 frames); None for other map sizes."""
    name = {(46, 46): "six_people", (46, 82): "twenty_720p"}.get((lh, lw))
    if name is None:
        return None
    d = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
    return np.concatenate([d["paf_low"], d["heat_low"]])


def optimal_size(h, w, size=368, stride=8):
    """compute_optimal_size (pose_detector.py:57-73): (net_w, net_h)."""
    if w < h:
        ow, oh = size, np.round(size * h / w)
    else:
        oh, ow = size, np.round(size * w / h)
    ow, oh = int(ow), int(oh)
    return ow + (-ow) % stride, oh + (-oh) % stride


def blas_info():
    try:
        from threadpoolctl import threadpool_info
        info = threadpool_info()
        blas = [i for i in info if i.get("user_api") == "blas"]
        if blas:
            return blas[0].get("internal_api", "?"), int(blas[0].get("num_threads", 1))
    except Exception:
        pass
    return "unknown", os.cpu_count() or 1


def cpu_baseline(frames, low_maps, n_frames):
    """The CPU restatement of the reference path on the host cores: oracle forward (Chainer's CPU
    conv: im2col + np.tensordot sgemm) + the NumPy/SciPy post-process (oracle/postproc_np.py, the
    reference's own library calls) on the same COCO-like maps; median per frame of n_frames after
    one warm-up (BASELINE.md CPU-baseline plan)."""
    from oracle import forward as F
    from oracle import cvresize
    from oracle import postproc_np as PN
    import importlib
    W = importlib.import_module(PKG + ".weights").random_weights(seed=0)
    vendor, threads = blas_info()

    def one(f):
        t0 = time.perf_counter()
        x = cvresize.preprocess(cvresize.resize_linear_u8(f, 368, 368))
        F.cocoposenet_forward(W, x)
        PN.postprocess(low_maps[:38], low_maps[38:], f.shape[0], f.shape[1])
        return time.perf_counter() - t0

    one(frames[0])  # warm-up
    times = [one(frames[(i + 1) % len(frames)]) for i in range(n_frames)]
    med = statistics.median(times)
    return {"value": round(1.0 / med, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": "median of %d frames after 1 warm-up (%.2f s/frame, %.1f s total): oracle forward "
                      "(im2col + np.tensordot sgemm, 368x368) + NumPy/SciPy post-process restatement "
                      "(oracle/postproc_np.py) on the 6-person maps" % (n_frames, med, sum(times)),
            "blas": vendor, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "nproc": os.cpu_count(),
            "cores_note": "BLAS threads = OMP_NUM_THREADS, which the GPU box sets to the host-CPU share it "
                          "allots one GPU (16); nproc counts every CPU of the shared machine"}


KERNEL_7X7 = {0: "conv_bf16x3<7", 1: "conv7_halo_bf16x3", 2: "conv7_halo_bf16x3", 3: "conv_halo_bf16x3<7",
              4: "conv_m16_bf16x3<7", 5: "conv_m16_bf16x3<7", 6: "conv_pair_bf16x3<7", 7: "conv_db_bf16x3<7",
              8: "conv_m16_bf16x3<7", 9: "conv_big_bf16x3<7", 10: "conv_big_bf16x3<7", 11: "conv_big_bf16x3<7"}
MFMA_7X7 = {4: "v_mfma_f32_16x16x32_bf16", 5: "v_mfma_f32_16x16x32_bf16", 6: "v_mfma_f32_16x16x32_bf16",
            8: "v_mfma_f32_16x16x32_bf16"}


def committed_traffic(kernel, workload, batch, precision, halo_mode, launch_ms=None):
    """HBM bytes per launch (read + write) of `kernel` from a committed rocprofv3 PMC summary
    (profiles/**/*_traffic.json: FETCH_SIZE x 2 -- every fabric read request is 128 B and FETCH_SIZE
    tallies it at 64 B, profiles/fetch_calib_r03.md -- + WRITE_SIZE, tools/summarize_profile.py)
    taken on this exact workload (same workload string, batch, precision and 7x7 kernel family).
    Among the matching sets: the newest round's, and within it the one whose average kernel time
    is closest to this run's launch_ms (round-5 tags ranked by letter count
    picked an older, slower set).  Returns (bytes, source, source_avg_ms), (None, None, None)
    when none matches."""
    import glob
    cands = []
    for p in glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")) + \
            glob.glob(os.path.join(REPO, "profiles", "*", "*_traffic.json")):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        cfg = d.get("config") or {}
        if cfg.get("frames_per_step_per_gpu") != batch or d.get("precision", "bf16x3") != precision:
            continue
        if cfg.get("workload") and workload and cfg["workload"] != workload:
            continue
        if KERNEL_7X7.get(d.get("halo_mode", 1)) != KERNEL_7X7.get(halo_mode):  # same 7x7 kernel
            continue
        m = re.match(r"r(\d+)", os.path.basename(p))
        rnd = int(m.group(1)) if m else -1
        ks = {k.replace("op::", ""): v for k, v in d.get("kernels", {}).items()}
        # every instantiation of the 7x7 family, weighted by its launches (sets from round 6 on record
        # them): the roofline's launch_ms averages over all 7x7 launches too (C4 runs several tiles);
        # older sets: the named instantiation alone
        fam = [v for k, v in ks.items() if k.startswith(kernel.split(" ")[0]) and v.get("calls")]
        if not fam:
            fam = [dict(v, calls=1) for k, v in ks.items() if k.startswith(kernel)]
        if not fam:
            continue
        calls = sum(v["calls"] for v in fam)
        byts = sum((v["read_bytes"] + v["write_bytes"]) * v["calls"] for v in fam) / calls
        avg_ms = sum(float(v.get("avg_ns", 0.0)) * v["calls"] for v in fam) / calls * 1e-6
        dist = abs(avg_ms - launch_ms) / launch_ms if launch_ms and avg_ms > 0 else 0.0
        cands.append(((rnd, -dist), int(byts), os.path.relpath(p, os.path.join(REPO, "profiles")),
                      round(avg_ms, 4) or None))
    if not cands:
        return None, None, None
    best = max(cands, key=lambda c: c[0])
    return best[1], best[2], best[3]


class Runner(object):
    """One configuration's step loop on this rank: async uploads from a 2-batch pinned pool, the
    staged path (single scale or precise), and the step's results to the host.

    Device path (default, any N): after the post-process the step's per-frame result records are
    packed in HBM and gathered to rank 0 on a communicator stream (an RCCL communicator of one rank
    at N = 1), landing in pinned memory; the host collects step k-1's records while the GPU runs
    step k, so no per-step host synchronisation idles the GPU.  Host path (the labelled fallback
    when RCCL refuses the setup): synchronous op_fetch_results + the TCP gather."""

    def __init__(self, L, Fr, ctx, args, B, FH, FW, rank, world, gather):
        self.L, self.Fr, self.ctx, self.args, self.B = L, Fr, ctx, args, B
        self.rank, self.world, self.gather = rank, world, gather
        rng = np.random.default_rng(1234 + rank)
        self.pool = [L.PinnedFrames(B, FH, FW) for _ in range(2)]
        for p in self.pool:
            p.array[...] = rng.integers(0, 256, (B, FH, FW, 3), dtype=np.uint8)
        self.k = 0
        self.persons = 0
        self.over_caps = 0  # device-path frames not delivered whole (must stay 0: overflow frames are re-run)
        self.overflow = 0  # device-path frames delivered through the overflow message (re-run uncapped)
        # host path: the TCP fallback, detect_precise (full-resolution results), and workloads that
        # may exceed the batched post-process caps (fetch_results re-runs those frames uncapped)
        self.sync = not gather.device or bool(args.precise)
        self.pending = []  # collect flags of the gathers in flight (oldest first)
        self.ctx.upload_frames(self.pool[0].array)

    def step(self, collect):
        a, ctx, B = self.args, self.ctx, self.B
        if a.precise:
            ctx.run_staged_precise()
        else:
            ctx.run_staged(graph=bool(a.graph))
        base = self.k * B * self.world + self.rank
        if not self.sync:
            self.gather.g.submit(0, B, base, self.world)
            ctx.upload_frames(self.pool[(self.k + 1) % 2].array)  # next step's frames, overlapped
            self.pending.append(collect)
            if len(self.pending) == 2:  # collect step k-1's records (step k is in flight)
                self._collect()
        else:
            ctx.upload_frames(self.pool[(self.k + 1) % 2].array)
            ctx.synchronize()
            res = ctx.fetch_results(0, B)
            if collect:
                self.persons += sum(r[2].n_persons for r in res)
            if self.world > 1 and not self.gather.device:
                self.gather.g.submit([(base + i * self.world, r[2].status, r[2].n_peaks, r[0], r[1])
                                      for i, r in enumerate(res)])
                self.pending.append(False)
                if len(self.pending) == 2:
                    self.gather.g.wait()
                    self.pending.pop(0)
        self.k += 1

    def _collect(self):
        got = self.gather.g.wait(raw=True)  # collective: also ships every rank's overflow frames
        if self.pending.pop(0) and got is not None:  # rank 0: every rank's records of that step
            raw, overflow = got
            persons, missing = self.Fr.count_persons(raw, GATHER_PERSONS, overflow)
            self.persons += persons
            self.over_caps += missing
            self.overflow += len(overflow)

    def drain(self):
        while self.pending:
            if not self.sync:
                self._collect()
            else:
                self.gather.g.wait()
                self.pending.pop(0)

    def close(self):
        for p in self.pool:
            p.close()


class Gather(object):
    def __init__(self, g, device, label):
        self.g, self.device, self.label = g, device, label


def make_gather(Fr, ctx, transport, world):
    g, err = None, None
    try:
        g = Fr.RcclGather(ctx, transport, GATHER_PERSONS, timeout=300.0)
    except Exception as e:  # labelled, never silent: the line says which transport ran
        err = e
    if world > 1:
        # one transport for every rank: if the communicator came up on some ranks only, all of them
        # take the TCP gather (a rank left on RCCL would wait for peers that never join)
        failed = transport.all_reduce(0.0 if err is None else 1.0, "sum")
        if failed > 0 and g is not None:
            g.close()
            g, err = None, "%d rank(s) could not create the RCCL communicator" % int(failed)
    if g is not None:
        if world == 1:
            return Gather(g, True, "single GPU (results packed in HBM, copied to pinned memory on a side "
                                   "stream, collected one step behind)")
        return Gather(g, True, "frame-parallel x%d, RCCL ncclGather of per-frame result records from HBM to "
                               "rank 0" % world)
    if world == 1:
        return Gather(None, False, "single GPU (synchronous result fetch: RCCL unavailable: %s)" % err)
    return Gather(Fr.HostGather(transport, GATHER_PERSONS), False,
                  "frame-parallel x%d, TCP gather of result records (RCCL init failed: %s)" % (world, err))


def measure(run, ctx, transport, steps, warmup, prof_7x7):
    for _ in range(warmup):
        run.step(False)
    run.drain()
    ctx.synchronize()
    ctx.profile_classes(["conv7x7"])
    ctx.profile(prof_7x7)
    ctx.profile_reset()
    if transport:
        transport.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run.step(True)
    run.drain()
    ctx.synchronize()
    if transport:
        transport.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    return elapsed, prof


def batch1_line(L, ctx, low, FH, FW, steps=60, warmup=10):
    """Single-image latency (BASELINE config 2 "single 368x368 frame"; pose_detector.py:484-517 is a
    one-image call): per step ONE pinned u8 frame is uploaded, run through the whole path (resize +
    normalise, 92 convs, post-process on the staged 6-person maps) and its poses fetched to the host,
    synchronously -- eager launches and a replayed hipGraph.  ms_per_frame = wall time per call;
    the eager run also times the 7x7 launches with HIP events (frac of the 833 TF/s bf16x3 peak)
    and, over a few extra calls, every kernel class."""
    pinned = L.PinnedFrames(1, FH, FW)
    rng = np.random.default_rng(99)
    pinned.array[...] = rng.integers(0, 256, (1, FH, FW, 3), dtype=np.uint8)
    ctx.stage_frames(np.zeros((1, FH, FW, 3), np.uint8))
    if low is not None:
        ctx.stage_maps(np.ascontiguousarray(low[None]))
        ctx.use_staged_maps(True)
    out = {}
    try:
        for graph in (0, 1):
            def call():
                ctx.upload_frames(pinned.array)
                ctx.run_staged(graph=bool(graph))
                ctx.synchronize()
                return ctx.fetch_results(0, 1)
            for _ in range(warmup):
                call()
            ctx.profile_classes(["conv7x7"])
            ctx.profile(not graph)
            ctx.profile_reset()
            times = []
            for _ in range(steps):
                t0 = time.perf_counter()
                r = call()
                times.append(time.perf_counter() - t0)
            prof = ctx.profile_read()
            ctx.profile(False)
            key = "graph" if graph else "eager"
            med = statistics.median(times)
            line = {"ms_per_frame_median": round(med * 1e3, 4), "ms_per_frame_min": round(min(times) * 1e3, 4),
                    "frames_per_s": round(1.0 / med, 2), "persons": int(r[0][2].n_persons)}
            ms7, n7, fl7, _ = prof["conv7x7"]
            if not graph and n7 and ms7 > 0:
                line["conv7x7_ms"] = round(ms7 / steps, 4)
                line["conv7x7_frac_of_833"] = round(fl7 / (ms7 * 1e-3) / 1e12 / (BF16_DENSE_PEAK_TFLOPS / 3.0), 4)
            out[key] = line
        ctx.profile_classes(list(ctx.PROFILE_CLASSES))
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(10):
            ctx.upload_frames(pinned.array)
            ctx.run_staged()
            ctx.synchronize()
        pall = ctx.profile_read()
        ctx.profile(False)
        out["stage_ms_per_frame"] = {k: round(v[0] / 10, 4) for k, v in pall.items() if v[1]}
        L.conv_census(reset=True)
        ctx.upload_frames(pinned.array)
        ctx.run_staged()
        ctx.synchronize()
        cen = L.conv_census(reset=True)
        out["conv7x7_tiles"] = {"npx": cen["npx"], "splitk_launches": cen["7x7_splitk"], "m16q_launches": cen["7x7_q"]}
        out["note"] = ("one %dx%d frame per synchronous call: upload, run_staged, fetch_results; median of %d "
                       "calls after %d warm-up" % (FW, FH, steps, warmup))
    finally:
        ctx.use_staged_maps(False)
        pinned.close()
    return out


def bench_line(args, L, Wm, Fr, transport, rank, world, local):
    """One configuration (args.frame / args.precise / args.batch) on this rank: context, gather and
    step loop, the timed steps, the per-class breakdown and the roofline; returns the JSON fields
    and the live state (close_line frees it)."""
    FH, FW = (int(v) for v in args.frame.lower().split("x"))
    headline = (FH, FW) == (368, 368) and not args.precise
    if args.batch is None:  # three rounds of full-chip 7x7 launches per step (single scale); C4: 16 frames
        args.batch = 16 if args.precise else (232 if (FH, FW) == (368, 368) else 64)
    B = args.batch
    net_w, net_h = optimal_size(FH, FW)
    halo_mode = int(os.environ.get("OP_HALO_MODE", "4"))
    limits = L.OpLimits()
    limits.max_batch = B
    ctx = L.Context(local, None, limits)
    ctx.set_precision(args.precision)
    ctx.set_weights(Wm.random_weights(seed=0))
    low = golden_maps(net_h // 8, net_w // 8) if not args.precise else golden_maps(46, 82)
    if low is None:
        args.maps = "network"
    # the post-process input: staged COCO-like maps (the forward still runs in full and writes its
    # own), at the network map size (__call__) or upsampled to the frame size (detect_precise)
    ctx.stage_frames(np.zeros((B, FH, FW, 3), np.uint8))
    if args.maps == "synthetic":
        m = low if not args.precise else ctx.resize_images(low, FH, FW)
        ctx.stage_maps(np.ascontiguousarray(np.repeat(m[None], B, axis=0)))
        ctx.use_staged_maps(True)
    gather = make_gather(Fr, ctx, transport, world)
    run = Runner(L, Fr, ctx, args, B, FH, FW, rank, world, gather)
    elapsed, prof = measure(run, ctx, transport, args.steps, args.warmup,
                            not args.no_profile and not args.graph)
    persons = run.persons
    # per-class breakdown from a few extra (untimed) steps with every class evented
    ctx.profile_classes(list(ctx.PROFILE_CLASSES))
    ctx.profile(not args.no_profile)
    ctx.profile_reset()
    n_extra = 0 if args.no_profile else 3
    for _ in range(n_extra):
        run.step(False)
    run.drain()
    ctx.synchronize()
    prof_all = ctx.profile_read()
    ctx.profile(False)
    over_caps = run.over_caps
    if transport:
        elapsed = transport.all_reduce(elapsed, "max")
        persons = transport.all_reduce(float(persons), "sum")
        over_caps = transport.all_reduce(float(over_caps), "sum")

    frames_total = world * B * args.steps
    value = frames_total / elapsed
    ms7, n7, fl7, by7 = prof["conv7x7"]
    arith = "bf16x3: 3xBF16 split products, f32 accumulate" if args.precision == "bf16x3" else "exact f32 MFMA"
    workload = ("%dx%d frames, full PoseDetector.%s path (upload, resize+normalise, 92-conv CocoPoseNet in %s, "
                "PAF post-process), batch of %d frames per GPU per step"
                % (FW, FH, "detect_precise" if args.precise else "__call__", arith, B))
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
        # the 7x7 kernel this workload actually ran (launch census of one extra step)
        L.conv_census(reset=True)
        run.step(False)
        run.drain()
        ctx.synchronize()
        cen = L.conv_census(reset=True)
        if args.precision == "bf16x3" and cen["npx"]:
            kern = "conv_m16_bf16x3<7, %d> (7x7 stage convs, 3xBF16 split on v_mfma_f32_16x16x32_bf16)" % max(
                cen["npx"], key=cen["npx"].get)
        elif args.precision != "bf16x3" and cen["f32_lds"]:
            kern = "conv_f32_lds<7, 16> (7x7 stage convs, LDS halo, v_mfma_f32_32x32x2_f32)"
        traffic, tsrc, tsrc_ms = committed_traffic(kern.split(">")[0], workload, B, args.precision, halo_mode,
                                                   ms7 / n7)
        roofline = {"bound": "mfma", "kernel": kern,
                    "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": tsrc,
                    "traffic_source_launch_ms": tsrc_ms,
                    "launch_ms": round(ms7 / n7, 4), "flops_per_launch": fl7 / n7,
                    "algorithmic_bytes_per_launch": by7 / n7}
    stage_ms = {k: round(v[0] / n_extra, 3) for k, v in prof_all.items()} if n_extra else {}
    metric = METRIC if headline else "frames/sec end-to-end (CNN+PAF grouping) at %dx%d%s, 1/2/4/8 MI355X" % (
        FW, FH, " multi-scale (%s)" % "/".join(str(v) for v in PARAMS_SCALES) if args.precise else "")
    maps_desc = ("post-process fed COCO-like %s maps from the reference's label generators%s" % (
        "6-person" if (FH, FW) == (368, 368) else "20-person",
        " (upsampled to the frame size: the full-resolution post-process)" if args.precise else "")
        if args.maps == "synthetic" else "post-process fed the network's own last stage")
    out = {
        "metric": metric, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16x3 (hi/lo split operands, f32 accumulate)" if args.precision == "bf16x3" else "f32",
        "data": "synthetic: seeded uint8 %dx%d BGR frames from a 2-batch pinned host pool, uploaded every step "
                "inside the timed region (copy stream, overlapped with the previous step); random-init "
                "CocoPoseNet (He-normal); %s" % (FW, FH, maps_desc),
        "config": {"workload": workload,
                   "frames_per_step_per_gpu": B, "net_input": "%dx%d" % (net_w, net_h),
                   "heatmap": "%dx%d" % optimal_size(FH, FW, 320) if not args.precise else "%dx%d" % (FW, FH),
                   "maps": args.maps, "parallelism": gather.label},
        "persons_per_s": round(persons / elapsed, 2),
        "frames_over_caps": int(over_caps),  # device-record path: frames not delivered whole (0 by design)
        "frames_overflow": int(run.overflow),  # frames delivered whole through the overflow message
        "gflop_per_frame": round((sum(L.forward_flops(*precise_net(FH, FW, sc)) for sc in PARAMS_SCALES)
                                  if args.precise else L.forward_flops(net_h, net_w)) / 1e9, 2),
        "stage_ms_per_step": stage_ms,
        "stage_ms_sum": round(sum(stage_ms.values()), 3),
        "stage_ms_note": "HIP-event sums per kernel class over %d untimed profiled steps (every kernel the "
                         "step launches is in a class; the sum falls short of ms_per_step by the gaps "
                         "between kernels)" % n_extra,
        "roofline": roofline,
    }
    # the whole step against the same peak: every conv FLOP of the step / the step's wall time
    step_tf = out["gflop_per_frame"] * 1e9 * frames_total / elapsed / 1e12
    out["step_tflops"] = round(step_tf, 2)
    out["step_frac_of_peak"] = round(step_tf / (BF16_DENSE_PEAK_TFLOPS / 3.0 if args.precision == "bf16x3"
                                                else FP32_MATRIX_PEAK_TFLOPS), 4)
    return out, {"ctx": ctx, "run": run, "gather": gather, "low": low, "B": B, "FH": FH, "FW": FW}


def close_line(st):
    st["run"].close()
    g = st["gather"]
    if g.g is not None and g.device:
        g.g.close()
    st["ctx"].close()


SIDE_KEYS = ("value", "unit", "metric", "ms_per_step", "steps", "warmup", "config", "gflop_per_frame",
             "persons_per_s", "frames_over_caps", "frames_overflow", "stage_ms_per_step", "stage_ms_sum",
             "roofline", "step_tflops", "step_frac_of_peak")


def side_line(args, frame, precise, L, Wm, Fr, transport, local):
    """Another BASELINE config measured by this same run (world 1): a fresh context of its own, the
    same step loop and fields as `python bench.py --frame FRAME [--precise]` (its default batch)."""
    a = argparse.Namespace(**vars(args))
    a.frame, a.precise, a.batch, a.maps, a.graph = frame, precise, None, "synthetic", 0
    a.no_variants = a.no_cpu_baseline = True
    a.steps = args.side_steps or args.steps
    t0 = time.perf_counter()
    o, st = bench_line(a, L, Wm, Fr, transport, 0, 1, local)
    close_line(st)
    line = {k: o[k] for k in SIDE_KEYS if k in o}
    line["wall_s"] = round(time.perf_counter() - t0, 2)  # setup (weights, arenas) + warm-up + timed + profiled steps
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per step per GPU; default 232 for the 368x368 headline, 64 for 1280x720 single "
                         "scale (756 7x7 workgroups, 2.95 rounds; 981-989 -> 991-995 frames/s over 63 in an "
                         "interleaved A/B, profiles/r03/ab_r03_c5_batch_63_64.log), 16 for --precise.  232: the 7x7 kernel's 640-pixel raster tiles, "
                         "232 x 2116 / 640 = 767.05 -> 768 per branch x 2 = 1536 workgroups = six full rounds of "
                         "one per CU (114 frames left 14 CUs idle in its third round); interleaved A/B "
                         "1818-1824 / 1827-1835 / 1847-1849 frames/s at 114 / 116 / 232, "
                         "profiles/r03/ab_r03_batch_114_116_232.log")
    ap.add_argument("--maps", choices=["synthetic", "network"], default="synthetic",
                    help="post-process input: COCO-like multi-person maps (default) or the random-weight "
                         "network's own last stage")
    ap.add_argument("--cpu-frames", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true", help="skip the network-maps / fp32 side lines")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--no-side-lines", action="store_true",
                    help="skip the C5 720p and C4 multi-scale lines of the default run (variants)")
    ap.add_argument("--side-steps", type=int, default=None, help="timed steps of each side line (default: --steps)")
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
        args.no_variants = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("OP_BENCH_DEVICE"):  # rehearsal aid: every rank on one device (RCCL then refuses
        local = int(os.environ["OP_BENCH_DEVICE"])  # the duplicate GPU and the labelled TCP gather runs)
    import importlib
    L = importlib.import_module(PKG + "._lib")
    Wm = importlib.import_module(PKG + ".weights")
    Fr = importlib.import_module(PKG + ".frames")
    transport = Fr.SocketTransport(rank, world, addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                                   timeout=300.0)  # world 1: no sockets; bootstrap of the 1-rank gather

    out, st = bench_line(args, L, Wm, Fr, transport, rank, world, local)
    ctx, run, gather, low, B = st["ctx"], st["run"], st["gather"], st["low"], st["B"]
    cpu_frames = None
    if not args.no_variants and world == 1:
        # side lines (not `value`): the same workload with the network's own maps, and in exact f32
        variants = {}
        vsteps = 5
        # the random network's own maps, on the same asynchronous device-record path as the headline:
        # frames past the batched post-process caps reach the host whole through the overflow
        # re-runs (op_comm_overflow_result), timed on their own
        ctx.use_staged_maps(False)
        ov0, ovs0 = run.overflow, gather.g.overflow_s if gather.device else 0.0
        ovc0 = gather.g.overflow_caps if gather.device else 0
        e, _ = measure(run, ctx, None, vsteps, 1, False)
        ovn = run.overflow - ov0
        ovs = (gather.g.overflow_s - ovs0) if gather.device else 0.0
        variants["maps_network"] = {
            "value": round(B * vsteps / e, 2), "ms_per_step": round(e / vsteps * 1e3, 3),
            "path": "device records (async)" if not run.sync else "synchronous fetch",
            "frames_overflow": ovn,
            "frames_over_caps_rerun": (gather.g.overflow_caps - ovc0) if gather.device else None,
            "overflow_ms_per_step": round(ovs / (vsteps + 1) * 1e3, 3),
            "note": "post-process on the random network's own last-stage maps (noise peaks); frames whose record "
                    "cannot carry the whole result travel as overflow: past 64 persons their rows are written "
                    "by the device into page-locked host memory when the records are packed, over the batched "
                    "caps they are re-run alone uncapped, on the host's collect path "
                    "(counted over the warm-up and timed steps)"}
        if args.maps == "synthetic":
            ctx.use_staged_maps(True)
        # exact f32 convolutions: the like-for-like arithmetic of the reference (Chainer fp32)
        ctx.set_precision("fp32")
        ctx.profile_classes(["conv7x7"])
        e, p32 = measure(run, ctx, None, vsteps, 1, True)
        ctx.profile_classes(list(ctx.PROFILE_CLASSES))
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(3):
            run.step(False)
        run.drain()
        ctx.synchronize()
        pall = ctx.profile_read()
        ctx.profile(False)
        ms, n, fl, _ = p32["conv7x7"]
        per_class = {}
        for k in ("conv7x7", "conv3x3", "conv1x1"):
            cms, cn, cfl, _ = pall[k]
            if cn and cms > 0:
                per_class[k] = {"ms_per_step": round(cms / 3, 3), "tflops": round(cfl / (cms * 1e-3) / 1e12, 2),
                                "frac_of_157.3": round(cfl / (cms * 1e-3) / 1e12 / FP32_MATRIX_PEAK_TFLOPS, 4)}
        variants["fp32"] = {"value": round(B * vsteps / e, 2), "ms_per_step": round(e / vsteps * 1e3, 3),
                            "dtype": "f32 (exact f32 MFMA, v_mfma_f32_32x32x2_f32)",
                            "conv7x7_frac_of_157.3_TFLOPs": round(fl / (ms * 1e-3) / 1e12 / FP32_MATRIX_PEAK_TFLOPS, 4)
                            if n else None,
                            "roofline_by_class": per_class,
                            "stage_ms_per_step": {k: round(v[0] / 3, 3) for k, v in pall.items()},
                            "stage_ms_note": "HIP-event sums per kernel class over 3 untimed profiled steps"}
        ctx.set_precision(args.precision)
        # single-image latency (BASELINE config 2 names one 368x368 frame): last, it re-stages
        variants["batch1"] = batch1_line(L, ctx, low, FH, FW)
        cpu_frames = run.pool[0].array[:4].copy()
        close_line(st)
        st = None
        # the other BASELINE configs on the same box in the same run (their own contexts): C5's 720p
        # stream shape, single scale (pose_detector.py:484-517), and C4's 4-scale detect_precise
        # (:433-482) on 1280x720 frames
        if not args.no_side_lines:
            variants["c5_720p"] = side_line(args, "720x1280", False, L, Wm, Fr, transport, local)
            variants["c4_precise"] = side_line(args, "720x1280", True, L, Wm, Fr, transport, local)
        out["variants"] = variants
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if cpu_frames is None:
            cpu_frames = run.pool[0].array[:4].copy()
        out["cpu_baseline"] = cpu_baseline(cpu_frames, low, args.cpu_frames)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if st is not None:
        close_line(st)
    if transport:
        transport.close()


if __name__ == "__main__":
    main()
