"""Frame-parallel path (frames.py) on the CPU, world size 2 and 3, no PyTorch: round-robin
sharding, the fixed-size result records, the socket transport's gather / broadcast / barrier /
max-reduce, and the per-rank timeout (a stalled rank fails the others loudly instead of hanging
them).  Per-frame compute here is the CPU oracle (test only); the device records + RCCL path is
tests/test_gpu_gather.py."""
import multiprocessing as mp
import os
import socket
import sys
import time

import numpy as np
import pytest

from conftest import REPO, golden_cases, load_golden, pkg_module

MAXP = 8  # smaller than the 20-person golden: those frames travel whole as overflow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame_results(ids):
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


def _worker(rank, world, port, n_frames, steps, q):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from importlib import import_module
    F = import_module("chainer_realtime_multi-person_pose_estimation_amd.frames")
    t = F.SocketTransport(rank, world, port=port, timeout=60)
    g = F.HostGather(t, MAXP)
    got = []
    for s in range(steps):  # the bench's pattern: submit step s, collect it at the end of step s+1
        ids = [s * n_frames + i for i in F.shard(n_frames, rank, world)]
        g.submit(_frame_results(ids))
        if s > 0:
            got.append(g.wait())
    got.append(g.wait())
    t.barrier()
    mx = t.all_reduce(float(rank + 1), "max")
    sm = t.all_reduce(1.0, "sum")
    if rank == 0:
        q.put((got, mx, sm))
    t.close()


@pytest.mark.parametrize("world,n_frames", [(2, 7), (3, 8)])
def test_socket_gather_matches_single_process(world, n_frames):
    F = pkg_module("frames")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, mx, sm = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == world and sm == world
    for s in range(steps):
        want = _frame_results(range(s * n_frames, (s + 1) * n_frames))  # every frame whole
        assert any(len(w[4]) > MAXP for w in want)  # some frames hold more persons than a record carries
        assert [r[0] for r in got[s]] == list(range(s * n_frames, (s + 1) * n_frames))
        for a, b in zip(got[s], want):
            assert a[:3] == b[:3] and np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])


def test_records_round_trip_and_person_cap():
    F = pkg_module("frames")
    res = _frame_results(range(5))
    back = F.unpack_records(F.pack_records(res, MAXP), MAXP)
    for (fid, st, npk, poses, scores), b in zip(res, back):
        k = min(len(scores), MAXP)
        assert b[0] == fid and b[1] == st and b[2] == npk
        assert np.array_equal(b[3], poses[:k]) and np.array_equal(b[4], scores[:k])
    assert F.record_bytes(64) == 32 + 64 * 55 * 8


def _stalled_worker(rank, port, q):
    sys.path.insert(0, REPO)
    from importlib import import_module
    F = import_module("chainer_realtime_multi-person_pose_estimation_amd.frames")
    t = F.SocketTransport(rank, 2, port=port, timeout=2.0)
    if rank == 1:
        time.sleep(6)  # stalls: never joins the gather
        t.close()
        return
    t0 = time.monotonic()
    try:
        t.gather(b"x")
        q.put(("no error", 0.0))
    except TimeoutError as e:
        q.put((str(e), time.monotonic() - t0))
    t.close()


def test_gather_times_out_on_a_stalled_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stalled_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msg, dt = q.get(timeout=60)
    for p in procs:
        p.join(timeout=30)
    assert "timed out" in msg and dt < 5.0, (msg, dt)


def test_count_persons_reads_exact_header_counts():
    """frames.count_persons (bench.py's device-record path): exact n_persons from the headers even
    past max_persons, zero for failed frames, over-cap frames (status 3) counted apart."""
    F = pkg_module("frames")
    rng = np.random.default_rng(0)
    recs = []
    for i in range(9):
        k = int(rng.integers(0, 7))
        status = 3 if i == 4 else 0
        recs.append((i, status, 40, rng.random((k, 18, 3)), rng.random(k)))
    buf = F.pack_records(recs, 4).tobytes()
    want = sum(len(r[4]) for r in recs if r[1] == 0)
    assert F.count_persons(buf, 4) == (want, 1)


def test_count_persons_and_merge_with_overflow():
    """A record over the batched caps (status 3, no persons) is counted from its overflow result;
    without one it counts as undelivered.  Records past max_persons keep their exact header count."""
    F = pkg_module("frames")
    res = _frame_results(range(4))
    rec = [(fid, st, npk, p, s) for fid, st, npk, p, s in res]
    rec[2] = (rec[2][0], F.STATUS_CAPACITY, rec[2][2], np.zeros((0, 18, 3)), np.zeros(0))
    buf = F.pack_records(rec, MAXP).tobytes()
    total = sum(len(r[4]) for r in res)
    assert F.count_persons(buf, MAXP, [res[2]]) == (total, 0)
    assert F.count_persons(buf, MAXP) == (total - len(res[2][4]), 1)
    merged = F.merge_overflow(F.unpack_records(buf, MAXP), [res[2]])
    assert merged[2][1] == 0 and np.array_equal(merged[2][4], res[2][4])
    back = F.unpack_full(F.pack_full(res))
    for a, b in zip(back, res):
        assert a[:3] == b[:3] and np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])


def _make_gather_rank(rank, world, port, q):
    """bench.make_gather with an RCCL communicator that comes up on rank 0 only (stand-in)."""
    try:
        sys.path.insert(0, REPO)
        import bench
        Fr = pkg_module("frames")
        closed = []

        class FakeRccl(object):
            def __init__(self, ctx, transport, max_persons, timeout=0.0):
                if transport.rank != 0:
                    raise RuntimeError("ncclCommInitRankConfig failed (test stand-in)")

            def close(self):
                closed.append(True)

        Fr.RcclGather = FakeRccl
        t = Fr.SocketTransport(rank, world, port=port, timeout=30.0)
        g = bench.make_gather(Fr, None, t, world)
        q.put((rank, type(g.g).__name__, g.device, bool(closed), "TCP gather" in g.label))
        t.close()
    except Exception as e:  # reported to the parent
        q.put((rank, "error", repr(e)))


def test_bench_gather_transport_is_one_for_all_ranks():
    """A communicator that comes up on some ranks only: every rank takes the labelled TCP gather and
    the ranks that had RCCL close it (bench.make_gather), instead of a split transport that hangs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_make_gather_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert got == [(0, "HostGather", False, True, True), (1, "HostGather", False, False, True)], got


def _lost_worker(rank, world, port, q):
    """One step of RcclGather.wait's host side on each rank: records of this rank's frames (rank 1's first
    frame is one that no keep slot held), then the overflow
    exchange -- the lost frame travels as a status, no rank raises before the collective."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from importlib import import_module
    F = import_module("chainer_realtime_multi-person_pose_estimation_amd.frames")
    t = F.SocketTransport(rank, world, port=port, timeout=60)
    ids = [i for i in F.shard(6, rank, world)]
    res = _frame_results(ids)
    own = []
    if rank == 1:
        fid, _, npk, _, _ = res[0]
        own = [(fid, F.STATUS_CAPACITY, npk, np.empty((0, 18, 3)), np.empty(0))]
    recs = F.pack_records(res, MAXP)
    got = t.gather(recs.tobytes())
    ovf = F.exchange_overflow(t, own)
    t.barrier()  # every rank got past the exchange
    if rank == 0:
        raw = b"".join(got)
        q.put((F.count_persons(raw, MAXP, ovf), [(r[0], r[1]) for r in ovf]))
    t.close()


def test_lost_keep_slot_frame_travels_as_status():
    """Advisor r04 (medium): a frame that no keep slot held is reported through the overflow exchange
    as status OP_ERR_CAPACITY (counted as not delivered), instead of an exception on its rank before
    the exchange that would leave the other ranks blocked in it."""
    F = pkg_module("frames")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lost_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    (persons, missing), ovf = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert missing == 1 and len(ovf) == 1 and ovf[0][1] == F.STATUS_CAPACITY
    assert persons > 0
