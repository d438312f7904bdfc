"""Synthetic DBoW2 vocabularies in the reference's text format (TemplatedVocabulary::saveToTextFile,
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1429-1449).  ORBvoc.txt is not shipped with the
reference, so the parity cases build trees of the same shape (k children per node,
L levels) whose node descriptors descend from their parent's by bit flips, with idf-like leaf
weights (some stopped at 0), written exactly as saveToTextFile writes them: the header
"k L  scoring weighting", then per node "parent isLeaf d0 ... d31  weight" with endl."""
import numpy as np


def _flip(rng, d, nbits):
    bits = np.unpackbits(d)
    idx = rng.choice(256, size=nbits, replace=False)
    bits[idx] ^= 1
    return np.packbits(bits)


def make_vocab(path, k=10, L=4, seed=0, scoring=0, weighting=0, order="bfs", trailing_newline=True,
               stop_frac=0.05, early_leaf=0.0, dup_children=0.0):
    """Write a vocabulary file; returns the leaf descriptors (to draw features near words)."""
    rng = np.random.default_rng(seed)
    root = rng.integers(0, 256, 32, dtype=np.uint8)
    nodes = []          # (parent, depth, desc)
    children = {0: []}

    def add(parent, depth, desc):
        nodes.append((parent, depth, desc))
        nid = len(nodes)            # file line i -> node id i (root is 0)
        children[nid] = []
        children[parent].append(nid)
        return nid

    def kids(parent_desc, depth):
        out = []
        for c in range(k):
            if out and rng.random() < dup_children:
                out.append(out[-1].copy())      # equal descriptors: first child wins the tie
            else:
                out.append(_flip(rng, parent_desc, max(4, 48 >> depth)))
        return out

    # build the tree (ids in BFS or DFS preorder, parents always before children)
    if order == "bfs":
        frontier = [(0, 0, root)]
        while frontier:
            nxt = []
            for pid, depth, pd in frontier:
                if depth == L or (depth >= 2 and rng.random() < early_leaf):
                    continue
                for d in kids(pd, depth):
                    nid = add(pid, depth + 1, d)
                    nxt.append((nid, depth + 1, d))
            frontier = nxt
    else:
        stack = [(0, 0, root)]
        while stack:
            pid, depth, pd = stack.pop()
            if depth == L or (depth >= 2 and rng.random() < early_leaf):
                continue
            ds = kids(pd, depth)
            ids = [add(pid, depth + 1, d) for d in ds]
            for nid, d in reversed(list(zip(ids, ds))):
                stack.append((nid, depth + 1, d))
    lines = [f"{k} {L}  {scoring} {weighting}"]
    leaves = []
    for i, (pid, depth, d) in enumerate(nodes, start=1):
        leaf = len(children[i]) == 0
        w = 0.0
        if leaf:
            leaves.append(d)
            w = 0.0 if rng.random() < stop_frac else float(rng.uniform(0.3, 9.0))
        ws = f"{w:g}"                       # ostream default precision (6 significant digits)
        lines.append(f"{pid} {1 if leaf else 0} " + " ".join(str(int(b)) for b in d) + "  " + ws)
    text = "\n".join(lines) + ("\n" if trailing_newline else "")
    with open(path, "w") as f:
        f.write(text)
    return np.array(leaves, np.uint8)


def features_near(leaves, n, seed=0, noise_bits=10):
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, len(leaves), n)
    return np.array([_flip(rng, leaves[p], noise_bits) for p in pick], np.uint8)


def tiny_vocab(path, trailing_newline=False):
    """k=2, L=2 by hand: root -> A (0x00.., internal), B (0xff.., internal);
    A -> a1 (0x00.., w 1.5), a2 (0x0f.., w 2); B -> b1 (0xf0.., w 0 = stopped), b2 (0xff.., w 0.5)."""
    z, o = [0] * 32, [255] * 32
    rows = [(0, 0, z, 0), (0, 0, o, 0), (1, 1, z, 1.5), (1, 1, [15] * 32, 2), (2, 1, [240] * 32, 0),
            (2, 1, o, 0.5)]
    lines = ["2 2  0 0"] + [f"{p} {l} " + " ".join(map(str, d)) + f"  {w:g}" for p, l, d, w in rows]
    with open(path, "w") as f:
        f.write("\n".join(lines) + ("\n" if trailing_newline else ""))
