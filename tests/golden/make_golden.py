"""Generate the post-process golden fixtures from the REFERENCE's own code.

Run in the build container only (it needs /root/reference, which does not exist on the GPU
box):  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

* Imports /root/reference/pose_detector.py and coco_data_loader.py with empty stub modules for
  the absent cv2 / chainer / pycocotools (nothing from them is called on the post-process path).
* Synthesises COCO-like network-resolution maps with the reference's own label generators
  (coco_data_loader.py:216-268) from synthetic skeletons.
* Upsamples them with the oracle's restatement of Chainer's F.resize_images
  (pose_detector.py:501-502; Chainer absent, parity unpinned at that one op) and runs the
  reference's unmodified compute_peaks_from_heatmaps (CPU branch) / compute_connections /
  grouping_key_points / subsets_to_pose_array (pose_detector.py:75-265, 508-517).
* pafs are wrapped in an ndarray subclass that turns ``paf[0][[ys, xs]]`` (a list of index
  arrays, pose_detector.py:147) into a tuple index: the NumPy<1.23 semantics the code was
  written for.

Each case is written as tests/golden/<case>.npz (inputs + expected outputs, no code).
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def install_stubs():
    for name in ["cv2", "chainer", "chainer.cuda", "chainer.serializers", "chainer.functions",
                 "chainer.links", "chainer.links.caffe", "chainer.dataset", "pycocotools",
                 "pycocotools.coco"]:
        sys.modules[name] = types.ModuleType(name)
    ch = sys.modules["chainer"]
    ch.cuda = sys.modules["chainer.cuda"]
    ch.cuda.get_array_module = lambda *a: np
    ch.serializers = sys.modules["chainer.serializers"]
    ch.functions = sys.modules["chainer.functions"]
    ch.links = sys.modules["chainer.links"]
    ch.links.caffe = sys.modules["chainer.links.caffe"]
    ch.links.Convolution2D = lambda *a, **k: None

    class Chain(object):
        def __init__(self, **kw):
            pass

    ch.Chain = Chain
    ch.dataset = sys.modules["chainer.dataset"]
    ch.dataset.DatasetMixin = object
    sys.modules["pycocotools.coco"].COCO = object
    sys.path.insert(0, REF)


class LegacyIndexArray(np.ndarray):
    """paf[0][[ys, xs]] -> paf[0][(ys, xs)] (NumPy < 1.23 list-of-arrays indexing)."""

    def __getitem__(self, key):
        if isinstance(key, list) and len(key) > 0 and all(isinstance(k, np.ndarray) for k in key):
            key = tuple(key)
        return np.ndarray.__getitem__(self, key)


# Synthetic standing-person template in body-height units (JointType order, entity.py:9-46).
TEMPLATE = np.array([
    [0.00, -0.90], [0.00, -0.70], [-0.22, -0.68], [-0.30, -0.40], [-0.32, -0.15],
    [0.22, -0.68], [0.30, -0.40], [0.32, -0.15], [-0.12, -0.10], [-0.14, 0.35],
    [-0.15, 0.80], [0.12, -0.10], [0.14, 0.35], [0.15, 0.80], [-0.04, -0.95],
    [0.04, -0.95], [-0.09, -0.92], [0.09, -0.92]])


def make_poses(rng, n, H, W, height_range, missing=()):
    poses = []
    for i in range(n):
        h = rng.uniform(*height_range)
        cx = rng.uniform(0.2 * W, 0.8 * W) if n > 1 else W / 2
        cy = rng.uniform(0.45 * H, 0.55 * H) if n > 1 else H / 2
        jit = rng.normal(0, 0.015, TEMPLATE.shape)
        pts = (TEMPLATE + jit) * h + np.array([cx, cy])
        vis = np.full((18, 1), 2.0)
        for j in missing:
            if i == 0:
                vis[j] = 0
        inside = (pts[:, 0] >= 0) & (pts[:, 0] <= W - 1) & (pts[:, 1] >= 0) & (pts[:, 1] <= H - 1)
        vis[~inside] = 0
        poses.append(np.hstack([pts, vis]))
    return np.array(poses)


def synth_maps(loader, rng, H, W, poses, noise):
    img = np.zeros((H, W, 3), np.uint8)
    if len(poses):
        heat = loader.generate_heatmaps(img, poses, 1.0)
        paf = loader.generate_pafs(img, poses, 1.0)
    else:
        heat = np.zeros((19, H, W), np.float32)
        heat[18] = 1
        paf = np.zeros((38, H, W), np.float32)
    if noise:
        heat = heat + rng.normal(0, noise, heat.shape).astype(np.float32)
        paf = paf + rng.normal(0, noise, paf.shape).astype(np.float32)
    return paf.astype(np.float32), heat.astype(np.float32)


def run_reference(pd, paf_low, heat_low, orig_h, orig_w):
    from oracle import cvresize, postproc  # noqa: E402
    from entity import params  # the reference's own params
    map_w, map_h = cvresize.compute_optimal_size(orig_h, orig_w, params["heatmap_size"])
    # reference's own compute_optimal_size must agree
    ref_size = pd.compute_optimal_size(np.zeros((orig_h, orig_w, 3)), params["heatmap_size"])
    assert (int(ref_size[0]), int(ref_size[1])) == (map_w, map_h)
    pafs = postproc.resize_images(paf_low, map_h, map_w).view(LegacyIndexArray)
    heatmaps = postproc.resize_images(heat_low, map_h, map_w)
    out = {"map_w": map_w, "map_h": map_h, "orig_h": orig_h, "orig_w": orig_w}
    all_peaks = pd.compute_peaks_from_heatmaps(heatmaps)
    out["all_peaks"] = np.array(all_peaks, np.float64).reshape(-1, 5)
    if len(all_peaks) == 0:
        out["status"] = 1  # empty: (0,18,3) / (0,)
        return out
    conns = pd.compute_connections(pafs, all_peaks, map_w, params)
    out["conn"] = np.concatenate([c.reshape(-1, 3) for c in conns])
    out["conn_off"] = np.concatenate([[0], np.cumsum([len(c) for c in conns])]).astype(np.int64)
    try:
        subsets = pd.grouping_key_points(conns, all_peaks, params)
    except IndexError:
        out["status"] = 4
        return out
    out["subsets"] = subsets
    all_peaks[:, 1] *= orig_w / map_w
    all_peaks[:, 2] *= orig_h / map_h
    poses = pd.subsets_to_pose_array(subsets, all_peaks)
    out["poses"] = np.asarray(poses, np.float64)
    out["poses_shape"] = np.array(np.asarray(poses).shape, np.int64)
    out["scores"] = subsets[:, -2]
    out["status"] = 0
    return out


def main():
    sys.path.insert(0, REPO)
    install_stubs()
    import pose_detector  # the reference, from /root/reference
    import coco_data_loader
    pd = pose_detector.PoseDetector(model=object())
    loader = object.__new__(coco_data_loader.CocoDataLoader)
    rng = np.random.default_rng(20261015)

    cases = {}
    # (name, map H, map W, orig_h, orig_w, persons, height range (map px), missing joints of person 0, noise)
    specs = [
        ("one_person", 46, 46, 584, 584, 1, (30, 34), (), 0.01),
        ("six_people", 46, 46, 480, 480, 6, (14, 22), (), 0.01),
        ("twenty_720p", 46, 82, 720, 1280, 20, (12, 20), (), 0.01),
        ("portrait_four", 62, 46, 642, 482, 4, (18, 26), (), 0.01),
        ("neckless_merge", 46, 46, 480, 480, 2, (22, 26), (1,), 0.0),
        ("no_person", 46, 46, 480, 480, 0, (0, 0), (), 0.0),
        ("empty", 46, 46, 480, 480, 0, (0, 0), (), 0.0),
        ("noise_crowd", 46, 46, 480, 480, 12, (10, 30), (), 0.08),
    ]
    for name, H, W, oh, ow, n, hr, missing, noise in specs:
        poses = make_poses(rng, n, H, W, hr, missing) if n else np.zeros((0, 18, 3))
        paf_low, heat_low = synth_maps(loader, rng, H, W, poses, noise)
        if name == "no_person":
            # isolated single peaks of several joint types, no PAF support: peaks but no subsets
            heat_low[:] = 0
            heat_low[18] = 1
            for j, (y, x) in enumerate([(8, 8), (30, 12), (20, 38), (40, 40)]):
                heat_low[j * 3, y, x] = 1.0
        if name == "neckless_merge":
            # second person keeps a neck far away so the neck-less skeleton assembles from two halves
            pass
        ref = run_reference(pd, paf_low, heat_low, oh, ow)
        ref["paf_low"] = paf_low
        ref["heat_low"] = heat_low
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **ref)
        cases[name] = ref
        print("%-16s peaks=%4d conns=%4d persons=%s status=%d" % (
            name, len(ref["all_peaks"]), len(ref.get("conn", [])),
            ref["poses_shape"][0] if "poses_shape" in ref else "-", ref["status"]))
    # grouping_key_points overflow: a connection that touches 3 subsets raises IndexError in the
    # reference (pose_detector.py:197).  Search small random connection sets for one.
    from entity import params as ref_params
    found = None
    for trial in range(20000):
        npk = 12
        peaks = np.zeros((npk, 5))
        peaks[:, 0] = np.sort(rng.integers(0, 18, npk))
        peaks[:, 1:3] = rng.integers(0, 40, (npk, 2))
        peaks[:, 3] = rng.uniform(0.1, 1.0, npk)
        peaks[:, 4] = np.arange(npk)
        conns = []
        for l, (ja, jb) in enumerate(ref_params["limbs_point"]):
            ia = np.nonzero(peaks[:, 0] == ja)[0]
            ib = np.nonzero(peaks[:, 0] == jb)[0]
            rows = [[a, b, rng.uniform(0.1, 1.0)] for a in ia for b in ib if rng.uniform() < 0.7]
            conns.append(np.array(rows, np.float64).reshape(-1, 3))
        try:
            pd.grouping_key_points(conns, peaks, ref_params)
        except IndexError:
            found = (peaks, conns)
            break
    assert found is not None
    peaks, conns = found
    np.savez_compressed(os.path.join(HERE, "grouping_indexerror.npz"), all_peaks=peaks,
                        conn=np.concatenate(conns), conn_off=np.concatenate([[0], np.cumsum([len(c) for c in conns])]),
                        status=4, grouping_only=1)
    print("grouping_indexerror found at trial", trial)
    # SciPy's own gaussian_filter on one upsampled map (pins the Gaussian restatement alone)
    from scipy.ndimage import gaussian_filter
    from oracle import postproc
    c = cases["six_people"]
    up = postproc.resize_images(c["heat_low"][:1], 320, 320)
    g = np.stack([gaussian_filter(up[i], sigma=2.5) for i in range(1)])
    np.savez_compressed(os.path.join(HERE, "gauss_scipy.npz"), up=up, g=g)


if __name__ == "__main__":
    main()
