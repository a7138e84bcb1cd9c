"""Frame-parallel serving across GPUs (one process per GPU, no PyTorch).

``PoseDetector.__call__`` (pose_detector.py:484-517) keeps no cross-frame state, so a stream of
frames shards with no data-path collective: frame i goes to rank i % world, and each rank runs its
frames on its own device-resident replica.  The only exchange is a gather of fixed-size per-frame
result records to rank 0 (include/openpose_hip.h "Multi-GPU result gather"):

* ``RcclGather`` -- the product path: records packed on the device after the post-process and
  gathered by ``ncclGather`` straight from HBM on a communicator stream (gather.hip), double
  buffered so step k's gather overlaps step k+1's compute, with a per-rank timeout.
* ``HostGather`` -- the same records and control flow over TCP sockets from host memory (CPU
  tests, world size 2, and any rank without a GPU).

Every frame reaches rank 0 whole, like the reference's ``__call__`` returns every frame's poses: a
record carries at most ``max_persons`` persons and no persons for a frame over the batched
post-process caps, so each rank also ships the whole results of its own such frames ("overflow",
re-run on its device from the post-process input the library kept aside, op_comm_overflow*) over
the TCP transport, and rank 0 merges them into the gathered records.

``SocketTransport`` is the small TCP star (rank 0 = hub) both use for bootstrap (RCCL's unique id),
barriers and scalar max-reductions; every receive has a timeout, so a stalled rank fails loudly
(``TimeoutError``) instead of hanging the job (SURVEY §5 failure detection).
"""
import os
import socket
import struct
import time

import numpy as np

N_JOINTS = 18
STATUS_CAPACITY = 3  # OP_ERR_CAPACITY (include/openpose_hip.h): the frame exceeded the batched caps
HDR_BYTES = 32  # int32 status, n_peaks, n_persons, 0; int64 frame id; 8 pad


def shard(n_frames, rank, world):
    """Frame ids owned by `rank` (round-robin)."""
    return list(range(rank, n_frames, world))


def record_bytes(max_persons):
    return HDR_BYTES + max_persons * (N_JOINTS * 3 + 1) * 8


def pack_records(results, max_persons):
    """Host-side records, byte-identical to the device's pack_records (runtime.hip).
    results: [(frame_id, status, n_peaks, poses (P,18,3), scores (P,))] -> (n, record_bytes) uint8."""
    rb = record_bytes(max_persons)
    out = np.zeros((len(results), rb), np.uint8)
    for i, (fid, status, n_peaks, poses, scores) in enumerate(results):
        n_persons = len(scores) if status == 0 else 0
        k = min(n_persons, max_persons)
        hdr = np.frombuffer(struct.pack("<iiiiqq", int(status), int(n_peaks), int(n_persons), 0, int(fid), 0), np.uint8)
        out[i, :HDR_BYTES] = hdr
        body = np.zeros(max_persons * (N_JOINTS * 3 + 1), np.float64)
        body[:k * N_JOINTS * 3] = np.asarray(poses, np.float64)[:k].reshape(-1)
        body[max_persons * N_JOINTS * 3:max_persons * N_JOINTS * 3 + k] = np.asarray(scores, np.float64)[:k]
        out[i, HDR_BYTES:] = body.view(np.uint8)
    return out


def unpack_records(buf, max_persons):
    """(n, record_bytes) uint8 (or raw bytes) -> [(frame_id, status, n_peaks, poses, scores)] in
    frame-id order; frames carry at most max_persons persons (status/n_peaks always exact)."""
    rb = record_bytes(max_persons)
    a = np.frombuffer(buf, np.uint8).reshape(-1, rb) if not isinstance(buf, np.ndarray) else buf.reshape(-1, rb)
    out = []
    for row in a:
        status, n_peaks, n_persons, _, fid, _ = struct.unpack("<iiiiqq", row[:HDR_BYTES].tobytes())
        body = row[HDR_BYTES:].view(np.float64)
        k = min(n_persons, max_persons)
        poses = body[:k * N_JOINTS * 3].reshape(k, N_JOINTS, 3).copy()
        scores = body[max_persons * N_JOINTS * 3:max_persons * N_JOINTS * 3 + k].copy()
        out.append((fid, status, n_peaks, poses, scores))
    out.sort(key=lambda r: r[0])
    return out


def pack_full(results):
    """Whole results of any person count (the overflow message): int32 n, int32 persons per record,
    then pack_records of them at that size."""
    mp = max([len(r[4]) for r in results if r[1] == 0] + [0])
    return struct.pack("<ii", len(results), mp) + pack_records(results, mp).tobytes()


def unpack_full(buf):
    n, mp = struct.unpack("<ii", bytes(buf[:8]))
    return unpack_records(bytes(buf[8:]), mp) if n else []


def exchange_overflow(transport, own):
    """The per-step overflow exchange (collective over the TCP transport): every rank's whole results
    of its frames that the records could not carry -- including frames no keep slot held, as status
    OP_ERR_CAPACITY -- to rank 0 (other ranks: None)."""
    if transport.world == 1:
        return own
    got = transport.gather(pack_full(own))
    return None if got is None else [r for g in got for r in unpack_full(g)]


def merge_overflow(records, overflow):
    """Records (unpacked) with the whole results of the overflow frames in place of theirs."""
    if not overflow:
        return records
    by_id = {r[0]: r for r in overflow}
    return [by_id.get(r[0], r) for r in records]


def count_persons(buf, max_persons, overflow=()):
    """(persons of every frame, frames still not delivered whole) of packed records plus the
    overflow results of the frames they could not carry.  Header person counts are exact even
    past max_persons; a frame over the batched caps counts its overflow result's persons (and
    counts as undelivered only when no overflow result came for it)."""
    rb = record_bytes(max_persons)
    a = np.frombuffer(buf, np.uint8).reshape(-1, rb)
    hdr = np.ascontiguousarray(a[:, :HDR_BYTES]).view(np.int32)  # status, n_peaks, n_persons, 0, id lo/hi
    fid = np.ascontiguousarray(a[:, 16:24]).view(np.int64).reshape(-1)
    ovf = {r[0]: r for r in overflow}
    persons, missing = 0, 0
    for i in range(len(a)):
        r = ovf.get(int(fid[i]))
        if r is not None:
            persons += len(r[4]) if r[1] == 0 else 0
            missing += r[1] == STATUS_CAPACITY  # no keep slot held it (RcclGather._own_overflow)
        elif hdr[i, 0] == 0:
            persons += int(hdr[i, 2])
        elif hdr[i, 0] == STATUS_CAPACITY:
            missing += 1
    return persons, missing


# ---------------------------------------------------------------- transport
def _recv_exact(sock, n):
    chunks, got = [], 0
    while got < n:
        b = sock.recv(min(n - got, 1 << 20))
        if not b:
            raise ConnectionError("peer closed the connection")
        chunks.append(b)
        got += len(b)
    return b"".join(chunks)


def _send_msg(sock, payload):
    sock.sendall(struct.pack("<q", len(payload)) + payload)


def _recv_msg(sock):
    (n,) = struct.unpack("<q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class SocketTransport(object):
    """TCP star of `world` ranks on one node: rank 0 listens on (addr, port), every other rank
    connects.  All operations are collective and time out after `timeout` seconds."""

    def __init__(self, rank, world, addr="127.0.0.1", port=None, timeout=120.0):
        self.rank, self.world, self.timeout = int(rank), int(world), float(timeout)
        self.peers = {}
        if self.world == 1:
            return
        port = int(port if port is not None else default_port())
        deadline = time.monotonic() + self.timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(self.timeout)
            try:
                while len(self.peers) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(self.timeout)
                    (r,) = struct.unpack("<i", _recv_exact(conn, 4))
                    self.peers[r] = conn
            except socket.timeout:
                raise TimeoutError("rank 0: only %d of %d ranks connected within %.0f s"
                                   % (len(self.peers) + 1, self.world, self.timeout))
            finally:
                srv.close()
        else:
            while True:
                try:
                    conn = socket.create_connection((addr, port), timeout=max(0.1, deadline - time.monotonic()))
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise TimeoutError("rank %d: rank 0 not reachable at %s:%d within %.0f s"
                                           % (self.rank, addr, port, self.timeout))
                    time.sleep(0.05)
            conn.settimeout(self.timeout)
            conn.sendall(struct.pack("<i", self.rank))
            self.peers[0] = conn

    def _io(self, fn, what):
        try:
            return fn()
        except socket.timeout:
            raise TimeoutError("rank %d: %s timed out after %.0f s (a rank stalled or died)"
                               % (self.rank, what, self.timeout))

    def gather(self, payload):
        """Rank 0: [payload of rank 0, 1, ...]; other ranks: None."""
        if self.world == 1:
            return [payload]
        if self.rank != 0:
            self._io(lambda: _send_msg(self.peers[0], payload), "gather")
            return None
        return [payload] + [self._io(lambda r=r: _recv_msg(self.peers[r]), "gather from rank %d" % r)
                            for r in range(1, self.world)]

    def broadcast(self, payload=None):
        """Rank 0's payload on every rank."""
        if self.world == 1:
            return payload
        if self.rank == 0:
            for r in range(1, self.world):
                self._io(lambda r=r: _send_msg(self.peers[r], payload), "broadcast")
            return payload
        return self._io(lambda: _recv_msg(self.peers[0]), "broadcast")

    def barrier(self):
        self.gather(b"")
        self.broadcast(b"" if self.rank == 0 else None)

    def all_reduce(self, value, op="max"):
        """max / sum of one float over ranks, on every rank."""
        got = self.gather(struct.pack("<d", float(value)))
        res = None
        if got is not None:
            vals = [struct.unpack("<d", g)[0] for g in got]
            res = struct.pack("<d", max(vals) if op == "max" else sum(vals))
        return struct.unpack("<d", self.broadcast(res))[0]

    def close(self):
        for c in self.peers.values():
            try:
                c.close()
            except OSError:
                pass
        self.peers = {}


def default_port():
    """Port of the transport's hub: OP_STORE_PORT, else MASTER_PORT + 101 (torchrun's own store
    holds MASTER_PORT), else 29611."""
    if os.environ.get("OP_STORE_PORT"):
        return int(os.environ["OP_STORE_PORT"])
    if os.environ.get("MASTER_PORT"):
        return (int(os.environ["MASTER_PORT"]) + 101) % 65536
    return 29611


# ---------------------------------------------------------------- gathers
class HostGather(object):
    """Result records gathered over the socket transport from host memory (CPU path)."""

    def __init__(self, transport, max_persons=64):
        self.t, self.max_persons = transport, int(max_persons)
        self.pending = []

    def submit(self, results):
        """results: this rank's [(frame_id, status, n_peaks, poses, scores)] of one step (whole
        results: the frames with more persons than a record holds travel as overflow)."""
        rec = pack_records(results, self.max_persons).tobytes()
        ovf = pack_full([r for r in results if r[1] == 0 and len(r[4]) > self.max_persons])
        self.pending.append(struct.pack("<q", len(rec)) + rec + ovf)

    def wait(self, timeout=None):
        """Rank 0: every rank's whole results of the oldest submitted step, by frame id; else None."""
        got = self.t.gather(self.pending.pop(0))
        if got is None:
            return None
        recs, ovf = [], []
        for g in got:
            (n,) = struct.unpack("<q", g[:8])
            recs.append(g[8:8 + n])
            ovf += unpack_full(g[8 + n:])
        return merge_overflow(unpack_records(b"".join(recs), self.max_persons), ovf)


class RcclGather(object):
    """Result records packed on the device and gathered to rank 0 by RCCL (gather.hip)."""

    def __init__(self, ctx, transport, max_persons=64, timeout=120.0):
        import ctypes
        from . import _lib
        self._lib, self._ct = _lib, ctypes
        self.ctx, self.t, self.max_persons, self.timeout = ctx, transport, int(max_persons), float(timeout)
        L = _lib.lib()
        uid = (ctypes.c_uint8 * _lib.OP_COMM_ID_BYTES)()
        if transport.rank == 0:
            _lib.check(L.op_comm_unique_id(uid), "op_comm_unique_id")
        raw = transport.broadcast(bytes(uid) if transport.rank == 0 else None)
        uid = (ctypes.c_uint8 * _lib.OP_COMM_ID_BYTES).from_buffer_copy(raw)
        h = ctypes.c_void_p()
        _lib.check(L.op_comm_create(ctx.h, transport.world, transport.rank, uid, self.timeout, ctypes.byref(h)),
                   "op_comm_create")
        self.h = h
        self._sub = []  # (frame_base, frame_stride) of the outstanding submits, oldest first
        self.overflow_s = 0.0  # host time spent on this rank's overflow frames (re-runs, row copies)
        self.overflow_caps = 0  # of them, frames over the batched caps (re-run uncapped)
        self.lost = 0  # of them, frames no keep slot held: status OP_ERR_CAPACITY in their result
        self.lost_msg = ""

    def submit(self, first, n, frame_base, frame_stride):
        """Enqueue the gather of this rank's staged frames [first, first+n) (global ids
        frame_base + i * frame_stride) behind the context's queued work; returns at once."""
        self._lib.check(self._lib.lib().op_comm_gather_results(self.h, self.ctx.h, int(first), int(n),
                                                               self.max_persons, int(frame_base),
                                                               int(frame_stride)), "op_comm_gather_results")
        self._sub.append((int(frame_base), int(frame_stride)))

    def _own_overflow(self, base, stride):
        """Whole results of this rank's frames of the step just waited for that its records could
        not carry (op_comm_overflow / op_comm_overflow_result: re-run uncapped on this device)."""
        ct, lib_, L = self._ct, self._lib, self._lib.lib()
        cnt = ct.c_int32()
        lib_.check(L.op_comm_overflow(self.h, self.ctx.h, None, None, 0, ct.byref(cnt)), "op_comm_overflow")
        if cnt.value == 0:
            return []
        idx = (ct.c_int32 * cnt.value)()
        why = (ct.c_int32 * cnt.value)()
        lib_.check(L.op_comm_overflow(self.h, self.ctx.h, idx, why, cnt.value, ct.byref(cnt)), "op_comm_overflow")
        self.overflow_caps += sum(1 for w in why if w == 1)
        out = []
        for i in idx:
            cap = max(self.max_persons, 64)
            while True:
                poses = np.empty((cap, N_JOINTS, 3), np.float64)
                scores = np.empty(cap, np.float64)
                res = lib_.OpFrameResult()
                rc = L.op_comm_overflow_result(self.h, self.ctx.h, int(i), lib_.ptr(poses), lib_.ptr(scores), cap,
                                               ct.byref(res))
                if rc == lib_.OP_ERR_CAPACITY and res.n_persons > cap:
                    cap = res.n_persons
                    continue
                break
            if rc == lib_.OP_ERR_CAPACITY and res.status != lib_.OP_ERR_CAPACITY:
                # no keep slot held this frame (more overflow frames than slots in one gather; the
                # library grows the slots for the next packs): it travels as a frame status through
                # the exchange below -- an exception here would leave the other ranks waiting in it.
                # (A re-run whose own frame status is OP_ERR_CAPACITY is not a lost frame: its status
                # travels below like any other -- advisor r05)
                self.lost += 1
                self.lost_msg = lib_.last_error()
                out.append((base + int(i) * stride, STATUS_CAPACITY, int(res.n_peaks),
                            np.empty((0, N_JOINTS, 3)), np.empty(0)))
                continue
            if rc != lib_.OP_OK and rc != res.status:  # a frame status (e.g. the reference's IndexError) travels
                lib_.check(rc, "op_comm_overflow_result")
            k = res.n_persons if res.status == 0 else 0
            out.append((base + int(i) * stride, int(res.status), int(res.n_peaks), poses[:k].copy(), scores[:k].copy()))
        return out

    def wait(self, timeout=None, raw=False):
        """Rank 0: every rank's whole results of the oldest submitted step (unpacked and merged, by
        frame id; or (raw record bytes, overflow results) with raw=True); other ranks: None.
        Collective: every rank calls it once per submit (the overflow exchange is a TCP gather)."""
        ct = self._ct
        p, nf, rb = ct.c_void_p(), ct.c_int32(), ct.c_int64()
        # op_comm_wait dequeues the oldest slot even when it then fails (timeout, HIP error): pop the
        # matching submit first, so this FIFO and the C slot FIFO stay in step
        base, stride = self._sub.pop(0) if self._sub else (0, 1)
        self._lib.check(self._lib.lib().op_comm_wait(self.h, float(timeout or self.timeout), ct.byref(p),
                                                     ct.byref(nf), ct.byref(rb)), "op_comm_wait")
        t0 = time.perf_counter()
        own = self._own_overflow(base, stride)
        self.overflow_s += time.perf_counter() - t0
        ovf = exchange_overflow(self.t, own)
        if not p.value:
            return None
        buf = ct.string_at(p.value, nf.value * rb.value)
        return (buf, ovf) if raw else merge_overflow(unpack_records(buf, self.max_persons), ovf)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self._lib.lib().op_comm_destroy(self.h)
            self.h = None
