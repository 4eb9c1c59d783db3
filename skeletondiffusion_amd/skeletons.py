"""Skeleton graphs that parameterise the sampler: joint-correlation (adjacency) matrices and
node types.  Only the data needed to build Sigma_N and the per-type weights is kept (the
reference's skeleton classes, src/data/skeleton/kinematic/*.py, are out of scope).

Nodes are the joints without the hip/root (if_consider_hip=False, the eval setting,
configs/config_eval/task/hmp.yaml:4); the root's limbs are replaced by a hip triangle
(e.g. h36m.py:89-97).  Node types: left/right twins share a type ('LKnee'/'RKnee' ->
'Knee', kinematic/base.py:58-70).  tests/test_skeletons.py checks every table against the
adjacency, node types and names captured from the reference (tests/golden/cov_*.npz).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

# joint names WITH the root at index 0, limbs in that indexing, and the hip-triangle joints
_H36M17 = (
    ["GlobalRoot", "RHip", "RKnee", "RAnkle", "LHip", "LKnee", "LAnkle", "Torso", "Neck", "Nose", "Head",
     "LShoulder", "LElbow", "LWrist", "RShoulder", "RElbow", "RWrist"],
    [(0, 1), (0, 4), (1, 2), (2, 3), (4, 5), (5, 6), (0, 7), (7, 8), (8, 9), (9, 10), (8, 11), (8, 14),
     (11, 12), (12, 13), (14, 15), (15, 16)],
    ("RHip", "LHip", "Torso"),
)

_AMASS22_NAMES = ["GlobalRoot", "LHip", "RHip", "Spine1", "LKnee", "RKnee", "Spine3", "LHeel", "RHeel", "Neck",
                  "LFoot", "RFoot", "BMN", "LSI", "RSI", "Head", "LShoulder", "RShoulder", "LElbow", "RElbow",
                  "LWrist", "RWrist"]
_AMASS22_LIMBS = [(0, 3), (3, 6), (6, 9), (9, 12), (12, 15), (9, 14), (14, 17), (17, 19), (19, 21), (9, 13),
                  (13, 16), (16, 18), (18, 20), (0, 2), (2, 5), (5, 8), (8, 11), (0, 1), (1, 4), (4, 7), (7, 10)]


def _mano_hand(side: str, wrist: int, first: int):
    names, limbs = [], []
    for f, finger in enumerate(["index", "middle", "pinky", "ring", "thumb"]):
        base = first + 3 * f
        names += [f"{side}_{finger}{k}" for k in (1, 2, 3)]
        limbs += [(wrist, base), (base, base + 1), (base + 1, base + 2)]
    return names, limbs


_lh_n, _lh_l = _mano_hand("left", 20, 22)
_rh_n, _rh_l = _mano_hand("right", 21, 37)

_FREEMAN18 = (
    ["GlobalRoot", "LHip", "RHip", "LKnee", "RKnee", "LAnkle", "RAnkle", "Nose", "LEye", "REye", "LEar", "REar",
     "LShoulder", "RShoulder", "LElbow", "RElbow", "LWrist", "RWrist"],
    [(0, 1), (0, 2), (1, 3), (2, 4), (3, 5), (4, 6), (0, 7), (7, 8), (7, 9), (8, 10), (9, 11), (7, 12), (7, 13),
     (12, 14), (13, 15), (14, 16), (15, 17)],
    ("RHip", "LHip", "Nose"),
)

SKELETONS: Dict[str, Tuple[List[str], List[Tuple[int, int]], Tuple[str, str, str]]] = {
    "h36m16": _H36M17,
    "amass21": (_AMASS22_NAMES, _AMASS22_LIMBS, ("LHip", "RHip", "Spine1")),
    "mano51": (_AMASS22_NAMES + _lh_n + _rh_n, _AMASS22_LIMBS + _lh_l + _rh_l, ("LHip", "RHip", "Spine1")),
    "freeman17": _FREEMAN18,
}


# hip-included variants (if_consider_hip=True, e.g. amass.py:81-83): the root joint is node 0 and
# the original limbs are kept (BASELINE config 3's "J=52" label for AMASS-MANO)
HIP_INCLUDED: Dict[str, str] = {"mano52": "mano51"}


def skeleton(key: str):
    """-> (node_names, node_limbs, adjacency (J,J) float32, node_types (J,) int64)."""
    if key in HIP_INCLUDED:
        names, limbs, _ = SKELETONS[HIP_INCLUDED[key]]
        nodes, node_limbs = list(names), [tuple(l) for l in limbs]
    else:
        names, limbs, (a, b, c) = SKELETONS[key]
        nodes = names[1:]
        idx = {n: i for i, n in enumerate(nodes)}
        node_limbs = [(idx[a], idx[b]), (idx[a], idx[c]), (idx[b], idx[c])]
        node_limbs += [(i - 1, j - 1) for i, j in limbs if i != 0 and j != 0]
    J = len(nodes)
    adj = np.zeros((J, J), dtype=np.float32)
    for i, j in node_limbs:
        adj[i, j] = adj[j, i] = 1.0
    stripped = [n[1:] if n[0] in "LR" and n[1].isupper() else n for n in nodes]
    uniq = list(dict.fromkeys(stripped))
    types = np.array([uniq.index(s) for s in stripped], dtype=np.int64)
    return nodes, node_limbs, adj, types
