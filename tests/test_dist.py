"""World-size-2 gloo rehearsal of the frame-parallel path (frames.py): round-robin sharding +
gather of fixed-size result records.  Per-frame compute here is the CPU oracle (test only)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import REPO, golden_cases, load_golden

MAXP = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame_results(ids):
    import sys
    sys.path.insert(0, REPO)
    from oracle import postproc as P
    cases = [c for c in golden_cases() if c != "noise_crowd"]
    out = []
    for fid in ids:
        d = load_golden(cases[fid % len(cases)])
        poses, scores = P.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
        poses = np.asarray(poses, np.float64).reshape(-1, 18, 3)
        out.append((fid, 0, len(d["all_peaks"]), poses, np.asarray(scores)))
    return out


def _worker(rank, world, port, n_frames, q):
    import sys
    sys.path.insert(0, REPO)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from importlib import import_module
    F = import_module("chainer_realtime_multi-person_pose_estimation_amd.frames")
    mine = F.shard(n_frames, rank, world)
    local = F.pack_records(_frame_results(mine), MAXP)
    allr = F.gather_records(local, MAXP)
    if rank == 0:
        q.put(allr)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_gather_matches_single_process():
    n_frames = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, REPO)
    from importlib import import_module
    F = import_module("chainer_realtime_multi-person_pose_estimation_amd.frames")
    want = F.pack_records(_frame_results(list(range(n_frames))), MAXP)
    assert got.shape == want.shape
    assert np.array_equal(got, want)
