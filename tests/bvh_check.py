"""Structure and SAH checks of a BVH in the reference's node encoding
(BVHNode_encoded, OpenglRayTracing/main.cpp:69-73: 12 f32 per node, dummy
node 0, root 1, child 0 = none, leaf iff n > 0, leaf triangles [index,
index + n) of the built order). Vectorised numpy, so million-triangle trees
check in about a second."""
from __future__ import annotations

import numpy as np


def tri_boxes(tris: np.ndarray):
    p = np.asarray(tris, np.float32).reshape(-1, 36)[:, :9].reshape(-1, 3, 3)
    return p.min(axis=1), p.max(axis=1)


def box_area(lo, hi):
    d = np.maximum(hi - lo, 0.0).astype(np.float64)
    return 2.0 * (d[:, 0] * d[:, 1] + d[:, 0] * d[:, 2] + d[:, 1] * d[:, 2])


def check_tree(tris: np.ndarray, nodes: np.ndarray, order: np.ndarray | None, leaf_size: int):
    """Asserts: a tree rooted at node 1 over every node, each triangle in exactly
    one leaf, leaves of 1..leaf_size triangles, every box the exact union of its
    triangles' boxes (tris given in input order, order[i] = input index at built
    position i; order None = tris already in built order). Returns (internal, leaves)."""
    nodes = np.asarray(nodes, np.float32).reshape(-1, 12)
    m = nodes.shape[0]
    n = tris.reshape(-1, 36).shape[0]
    if order is None:
        order = np.arange(n)
    assert np.array_equal(np.sort(order), np.arange(n)), "order is not a permutation"
    ids = np.arange(m)
    cnt = nodes[:, 3].astype(np.int64)
    leaf = (cnt > 0) & (ids >= 1)
    internal = (cnt == 0) & (ids >= 1)
    L = nodes[:, 0].astype(np.int64)
    R = nodes[:, 1].astype(np.int64)
    # a tree: every node but the root is the child of exactly one internal node,
    # and children have larger ids (no cycles)
    kids = np.concatenate([L[internal], R[internal]])
    assert np.all(kids > 0), "internal node without two children"
    assert np.all(np.concatenate([L[internal], R[internal]]) > np.concatenate([ids[internal], ids[internal]]))
    seen = np.bincount(kids, minlength=m)
    assert seen[1] == 0 and np.all(seen[2:] == 1), "not a tree rooted at node 1"
    # leaves partition the built positions
    start = nodes[leaf, 4].astype(np.int64)
    c = cnt[leaf]
    assert np.all((c >= 1) & (c <= leaf_size)), f"leaf sizes {c.min()}..{c.max()}"
    cover = np.zeros(n + 1, np.int64)
    np.add.at(cover, start, 1)
    np.add.at(cover, start + c, -1)
    assert np.all(np.cumsum(cover)[:n] == 1), "leaves do not cover every position exactly once"
    # exact boxes: leaves from their triangles, internal nodes from their children
    lo, hi = tri_boxes(tris)
    lo, hi = lo[order], hi[order]
    srt = np.argsort(start)
    st = start[srt]
    llo = np.minimum.reduceat(lo, st, axis=0)
    lhi = np.maximum.reduceat(hi, st, axis=0)
    leaf_ids = ids[leaf][srt]
    assert np.array_equal(nodes[leaf_ids, 6:9], llo) and np.array_equal(nodes[leaf_ids, 9:12], lhi), \
        "leaf box is not its triangles' union"
    ii = ids[internal]
    assert np.array_equal(nodes[ii, 6:9], np.minimum(nodes[L[ii], 6:9], nodes[R[ii], 6:9])), "internal box lo"
    assert np.array_equal(nodes[ii, 9:12], np.maximum(nodes[L[ii], 9:12], nodes[R[ii], 9:12])), "internal box hi"
    return int(internal.sum()), int(leaf.sum())


def sah_cost(nodes: np.ndarray) -> float:
    """Surface-area cost relative to the root: sum over internal nodes of area,
    plus sum over leaves of area x triangles (unit traversal and test costs)."""
    nodes = np.asarray(nodes, np.float32).reshape(-1, 12)[1:]
    a = box_area(nodes[:, 6:9], nodes[:, 9:12])
    cnt = nodes[:, 3].astype(np.float64)
    cost = np.where(cnt > 0, a * cnt, a).sum()
    return float(cost / a[0])


def depth(nodes: np.ndarray) -> int:
    nodes = np.asarray(nodes, np.float32).reshape(-1, 12)
    d = np.zeros(nodes.shape[0], np.int64)
    d[1] = 1
    best = 1
    # children have larger ids than their parents (check_tree), so one pass in id order suffices
    for k in range(1, nodes.shape[0]):
        if nodes[k, 3] == 0:
            for c in (int(nodes[k, 0]), int(nodes[k, 1])):
                d[c] = d[k] + 1
                best = max(best, d[c])
    return best
