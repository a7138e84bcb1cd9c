"""Frame-parallel serving across GPUs (one process per GPU).

``PoseDetector.__call__`` (pose_detector.py:484-517) has no cross-frame state, so a stream of
frames shards with no data-path collective: frame i goes to rank i % world.  Each rank runs its
frames on its own device-resident replica; the only exchange is a gather of fixed-size
per-frame result records to rank 0 (torch.distributed all_gather: RCCL over xGMI with the
'nccl' backend on MI355X, gloo on CPU for tests).
"""
import numpy as np

N_JOINTS = 18
HDR = 4  # frame_id, status, n_persons, n_peaks


def shard(n_frames, rank, world):
    """Frame ids owned by `rank` (round-robin)."""
    return list(range(rank, n_frames, world))


def record_width(max_persons):
    return HDR + max_persons * (1 + N_JOINTS * 3)


def pack_records(results, max_persons):
    """results: list of (frame_id, status, n_peaks, poses (P,18,3), scores (P,)) -> (n, R) f64."""
    out = np.zeros((len(results), record_width(max_persons)), np.float64)
    for i, (fid, status, n_peaks, poses, scores) in enumerate(results):
        p = min(len(scores), max_persons)
        out[i, 0] = fid
        out[i, 1] = status
        out[i, 2] = p
        out[i, 3] = n_peaks
        out[i, HDR:HDR + p] = np.asarray(scores, np.float64)[:p]
        out[i, HDR + max_persons:HDR + max_persons + p * N_JOINTS * 3] = np.asarray(poses, np.float64)[:p].reshape(-1)
    return out


def unpack_record(row, max_persons):
    p = int(row[2])
    scores = row[HDR:HDR + p].copy()
    poses = row[HDR + max_persons:HDR + max_persons + p * N_JOINTS * 3].reshape(p, N_JOINTS, 3).copy()
    return int(row[0]), int(row[1]), int(row[3]), poses, scores


def gather_records(local, max_persons, device=None):
    """All ranks contribute (n_local, R) records; every rank receives all of them ordered by frame id.

    Ranks may hold different counts: each pads to the max with frame_id -1 rows."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    R = record_width(max_persons)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    m = int(max(int(c.item()) for c in counts))
    buf = np.full((m, R), -1.0, np.float64)
    buf[:local.shape[0]] = local
    t = torch.from_numpy(buf).to(device) if device is not None else torch.from_numpy(buf)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    allr = np.concatenate([o.cpu().numpy() for o in outs])
    allr = allr[allr[:, 0] >= 0]
    return allr[np.argsort(allr[:, 0], kind="stable")]
