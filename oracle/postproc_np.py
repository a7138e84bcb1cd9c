"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

A NumPy / SciPy restatement of the reference's CPU post-process (pose_detector.py:75-265 and the
F.resize_images upsample of :501-502), written to *cost* what the reference costs: the same
library calls (scipy.ndimage.gaussian_filter, shifted-map comparisons + np.nonzero, per-pair
np.linspace / np.dot line integrals, Python-list greedy assignment, row-wise subset grouping with
np.vstack / np.delete).  bench.py's cpu_baseline times it; tests/test_oracle_np.py holds it to the
C restatement (oracle/postproc.c) and the reference-generated goldens bit for bit.

The reference's GPU branch (cupy) is not restated: the parity target is its CPU branch.
"""
import itertools

import numpy as np
from scipy.ndimage import gaussian_filter

from .postproc import PARAMS, N_JOINTS


def resize_align_corners(x, out_h, out_w):
    """Chainer <= 6 F.resize_images on (C, H, W) f32: align-corners bilinear, f64 weights cast to
    f32, ((w1*x00 + w2*x01) + w3*x10) + w4*x11 in f32 (the restatement in oracle/postproc.c)."""
    x = np.asarray(x, np.float32)
    _, h, w = x.shape

    def axis(n_in, n_out):
        t = np.linspace(0.0, n_in - 1.0, n_out)
        lo = np.clip(np.floor(t).astype(np.int64), 0, n_in - 2)
        return t, lo, lo + 1

    v, v0, v1 = axis(h, out_h)
    u, u0, u1 = axis(w, out_w)
    du1, du0 = (u1 - u)[None, :], (u - u0)[None, :]
    dv1, dv0 = (v1 - v)[:, None], (v - v0)[:, None]
    w1, w2 = (du1 * dv1).astype(np.float32), (du0 * dv1).astype(np.float32)
    w3, w4 = (du1 * dv0).astype(np.float32), (du0 * dv0).astype(np.float32)
    top, bot = x[:, v0, :], x[:, v1, :]
    acc = w1 * top[:, :, u0] + w2 * top[:, :, u1]
    acc = acc + w3 * bot[:, :, u0]
    return acc + w4 * bot[:, :, u1]


def find_peaks(heatmaps, params=PARAMS):
    """compute_peaks_from_heatmaps, CPU branch (:75-110): rows [joint, x, y, score, id] (f64)."""
    rows = []
    for joint in range(len(heatmaps) - 1):
        smooth = gaussian_filter(heatmaps[joint], sigma=params["gaussian_sigma"])
        up, down = np.zeros(smooth.shape), np.zeros(smooth.shape)
        lf, rt = np.zeros(smooth.shape), np.zeros(smooth.shape)
        up[1:, :], down[:-1, :] = smooth[:-1, :], smooth[1:, :]
        lf[:, 1:], rt[:, :-1] = smooth[:, :-1], smooth[:, 1:]
        is_peak = np.logical_and.reduce((smooth > params["heatmap_peak_thresh"], smooth > up, smooth > down,
                                         smooth > lf, smooth > rt))
        ys, xs = np.nonzero(is_peak)
        for x, y in zip(xs, ys):
            rows.append((joint, x, y, smooth[y, x], len(rows)))
    return np.array(rows)


def _limb_candidates(paf_xy, peaks_a, peaks_b, img_len, params):
    """compute_candidate_connections (:135-159): [(id_a, id_b, score)] in the reference's order,
    then stably sorted by score, descending."""
    n = params["n_integ_points"]
    found = []
    for pa, pb in itertools.product(peaks_a, peaks_b):
        d = pb[:2] - pa[:2]
        length = np.linalg.norm(d)
        if length == 0:
            continue
        line = np.stack([np.linspace(pa[1], pb[1], num=n), np.linspace(pa[0], pb[0], num=n)]).T.round().astype("i")
        yy, xx = np.hsplit(line, 2)
        samples = np.hstack([paf_xy[0][yy, xx], paf_xy[1][yy, xx]])
        proj = np.dot(samples, d / length)
        score = proj.sum() / len(proj) + min(params["limb_length_ratio"] * img_len / length
                                             - params["length_penalty_value"], 0)
        if sum(proj > params["inner_product_thresh"]) > params["n_integ_points_thresh"] and score > 0:
            found.append([int(pa[3]), int(pb[3]), score])
    return sorted(found, key=lambda c: c[2], reverse=True)


def connect_limbs(pafs, all_peaks, img_len, params=PARAMS):
    """compute_connections (:161-181): per limb, greedy first-fit over the sorted candidates."""
    out = []
    for limb, (ja, jb) in enumerate(params["limbs_point"]):
        peaks_a = all_peaks[all_peaks[:, 0] == ja][:, 1:]
        peaks_b = all_peaks[all_peaks[:, 0] == jb][:, 1:]
        taken = np.zeros((0, 3))
        if len(peaks_a) and len(peaks_b):
            limit = min(len(peaks_a), len(peaks_b))
            for ia, ib, score in _limb_candidates(pafs[[2 * limb, 2 * limb + 1]], peaks_a, peaks_b, img_len, params):
                if ia in taken[:, 0] or ib in taken[:, 1]:
                    continue
                taken = np.vstack([taken, [ia, ib, score]])
                if len(taken) >= limit:
                    break
        out.append(taken)
    return out


def _add_joint(person, joint, peak, peaks, score):
    person[joint] = peak
    person[-1] += 1
    person[-2] += peaks[peak, 3] + score


def group_people(all_connections, peaks, params=PARAMS):
    """grouping_key_points (:183-250): (S, 20) subsets after the keep filter; IndexError where the
    reference raises it (a connection touching three subsets)."""
    people = -1 * np.ones((0, 20))
    for limb, conns in enumerate(all_connections):
        ja, jb = params["limbs_point"][limb]
        for a, b, score in conns[:, :3]:
            a, b = int(a), int(b)
            hits = [-1, -1]
            n_hits = 0
            for row, person in enumerate(people):
                if person[ja] == a or person[jb] == b:
                    hits[n_hits] = row  # a third hit raises IndexError, as in the reference
                    n_hits += 1
            if n_hits == 1:
                person = people[hits[0]]
                if person[jb] != b:
                    _add_joint(person, jb, b, peaks, score)
            elif n_hits == 2:
                p1, p2 = people[hits[0]], people[hits[1]]
                both = ((p1 >= 0).astype(int) + (p2 >= 0).astype(int))[:-2]
                if not np.any(both == 2):
                    p1[:-2] += p2[:-2] + 1
                    p1[-2:] += p2[-2:]
                    p1[-2:] += score
                    people = np.delete(people, hits[1], axis=0)
                else:
                    for p in (p1, p2):
                        if p[ja] == -1:
                            _add_joint(p, ja, a, peaks, score)
                        elif p[jb] == -1:
                            _add_joint(p, jb, b, peaks, score)
            elif n_hits == 0 and limb not in (9, 13):
                row = -1 * np.ones(20)
                row[ja], row[jb] = a, b
                row[-1] = 2
                row[-2] = sum(peaks[[a, b], 3]) + score
                people = np.vstack([people, row])
    keep = np.logical_and(people[:, -1] >= params["n_subset_limbs_thresh"],
                          people[:, -2] / people[:, -1] >= params["subset_score_thresh"])
    return people[keep]


def poses_of(people, all_peaks):
    """subsets_to_pose_array (:252-265)."""
    out = []
    for person in people:
        out.append(np.array([all_peaks[k][1:3].tolist() + [2] if k >= 0 else [0, 0, 0]
                             for k in person[:N_JOINTS].astype("i")]))
    return np.array(out)


def postprocess(paf_low, heat_low, orig_h, orig_w, params=PARAMS):
    """pose_detector.py:501-517 from the last-stage maps (38|19, h, w) of one frame."""
    from .cvresize import compute_optimal_size
    map_w, map_h = compute_optimal_size(orig_h, orig_w, params["heatmap_size"])
    pafs = resize_align_corners(paf_low, map_h, map_w)
    heat = resize_align_corners(heat_low, map_h, map_w)
    all_peaks = find_peaks(heat, params)
    if len(all_peaks) == 0:
        return np.empty((0, N_JOINTS, 3)), np.empty(0)
    people = group_people(connect_limbs(pafs, all_peaks, map_w, params), all_peaks, params)
    all_peaks[:, 1] *= orig_w / map_w
    all_peaks[:, 2] *= orig_h / map_h
    return poses_of(people, all_peaks), people[:, -2]
