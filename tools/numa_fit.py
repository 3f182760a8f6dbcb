#!/usr/bin/env python3
"""numa_fit.py -- which address bits decide whether an HBM address is near
XCC 0's or XCC 1's half of the chip (tools/numa_map output).

An address is "near 0" when the load from XCC 0 took fewer cycles than the
load from XCC 1 (same 256 B, a fresh line each).  Mode 0 (every 256 B of
32 MB): the run lengths of the near-0 / near-1 class and the bits that
explain it as an XOR of address bits.  Mode 1 (random bases, one bit flipped
at a time): per bit, how often flipping it flips the class.
usage: python3 tools/numa_fit.py gpurun_out/numa/map0.txt gpurun_out/numa/map1.txt
"""
import sys

import numpy as np


def load(path):
    a = np.loadtxt(path, comments="#", dtype=np.int64)
    return a[:, 0], a[:, 1], a[:, 2]


def mode0(path):
    off, l0, l1 = load(path)
    near0 = (l0 < l1).astype(np.int64)
    print(f"{path}: {len(off)} offsets, near XCC0 {near0.mean():.3f}; latency near {np.median(np.minimum(l0, l1)):.0f}, "
          f"far {np.median(np.maximum(l0, l1)):.0f} cycles; margin median {np.median(np.abs(l0 - l1)):.0f}")
    # runs
    ch = np.flatnonzero(np.diff(near0)) + 1
    runs = np.diff(np.concatenate([[0], ch, [len(near0)]])) * 256
    vals, cnt = np.unique(runs, return_counts=True)
    print("  run lengths (bytes: count):", dict(zip(vals.tolist()[:12], cnt.tolist()[:12])))
    # linear fit over GF(2): near0 = c ^ XOR of bits in S (bits 8..24)
    bits = list(range(8, 25))
    X = np.array([[(o >> b) & 1 for b in bits] + [1] for o in off], np.uint8)
    best = None
    # greedy: single bits and pairs of bits
    for i, b in enumerate(bits):
        for c in (0, 1):
            pred = (X[:, i] ^ c)
            acc = (pred == near0).mean()
            if best is None or acc > best[0]:
                best = (acc, (b,), c)
    for i in range(len(bits)):
        for j in range(i + 1, len(bits)):
            for c in (0, 1):
                pred = X[:, i] ^ X[:, j] ^ c
                acc = (pred == near0).mean()
                if acc > best[0]:
                    best = (acc, (bits[i], bits[j]), c)
    print(f"  best XOR fit: bits {best[1]} ^ {best[2]} explains {best[0]:.4f}")
    return near0


def mode1(path):
    off, l0, l1 = load(path)
    near0 = (l0 < l1).astype(np.int64)
    n = len(off) // 27
    flips = np.zeros(26)
    for k in range(n):
        base = near0[27 * k]
        for i in range(26):
            flips[i] += near0[27 * k + 1 + i] != base
    print(f"{path}: {n} bases; per bit (8..33) the fraction of flips that change the near side:")
    for i in range(26):
        print(f"  bit {8 + i:2d}: {flips[i] / n:.3f}")


def mode2(path):
    """16 lines per 4 KB page from each XCC: the page is near XCC 0 when its
    mean latency from XCC 0 is the lower.  Fits the side as an XOR of page
    address bits (12..33), exhaustively over subsets of up to 3 bits."""
    import itertools
    off, l0, l1 = load(path)
    pg = off >> 12
    order = np.argsort(pg, kind="stable")
    pg, l0, l1 = pg[order], l0[order], l1[order]
    pages, idx = np.unique(pg, return_index=True)
    m0 = np.add.reduceat(l0, idx) / np.diff(np.append(idx, len(pg)))
    m1 = np.add.reduceat(l1, idx) / np.diff(np.append(idx, len(pg)))
    near0 = (m0 < m1).astype(np.int64)
    margin = np.abs(m0 - m1)
    print(f"{path}: {len(pages)} pages, near XCC0 {near0.mean():.3f}, margin median {np.median(margin):.0f} "
          f"(p10 {np.percentile(margin, 10):.0f}) cycles")
    bits = list(range(12, 34))
    B = np.array([[(int(p) << 12 >> b) & 1 for b in bits] for p in pages], np.int64)
    best = (0, None, 0)
    for r in (1, 2, 3):
        for sub in itertools.combinations(range(len(bits)), r):
            x = np.bitwise_xor.reduce(B[:, list(sub)], axis=1)
            for c in (0, 1):
                acc = ((x ^ c) == near0).mean()
                if acc > best[0]:
                    best = (acc, tuple(bits[i] for i in sub), c)
    print(f"  best XOR of up to 3 page bits: {best[1]} ^ {best[2]} explains {best[0]:.4f}")
    seq = pages < 4096
    runs = np.diff(np.flatnonzero(np.diff(near0[seq]) != 0))
    print("  first 16 MB, run lengths in pages:", np.unique(runs, return_counts=True))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--mode2":
        mode2(sys.argv[2])
        sys.exit(0)
    mode0(sys.argv[1])
    if len(sys.argv) > 2:
        mode1(sys.argv[2])
