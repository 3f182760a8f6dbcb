"""Independent numpy restatement of the engine's synthetic workload definition.

Used by the golden-vector generator and the tests to produce the same source
bytes the device generator (storage-benchmarks_amd/csrc/rs_synth.h) writes, and
the same per-block erasure lists, without calling the engine.
"""
import numpy as np

M64 = (1 << 64) - 1


def mix64_int(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def mix64_np(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_row(seed: int, row: int, length: int) -> np.ndarray:
    """Bytes of synthetic row `row`: LE words mix(seed*phi + row*c + w)."""
    words = (length + 7) // 8
    base = (seed * 0x9E3779B97F4A7C15 + row * 0xD1B54A32D192ED03) & M64
    with np.errstate(over="ignore"):
        z = np.uint64(base) + np.arange(words, dtype=np.uint64)
    v = mix64_np(z)
    return v.view(np.uint8)[:length].copy()


def synth_block(seed: int, blk: int, k: int, length: int) -> np.ndarray:
    """[k][length] source rows of block `blk` (global rows blk*k .. blk*k+k-1)."""
    return np.stack([synth_row(seed, blk * k + j, length) for j in range(k)])


def erasure_pattern(seed: int, blk: int, k: int, e: int) -> np.ndarray:
    """e distinct originals of block `blk`, ascending (isa.cpp:137-153 procedure)."""
    chosen = set()
    ctr = 0
    s0 = mix64_int(seed ^ 0xA5A5A5A55A5A5A5A)
    while len(chosen) < e:
        r = s0 ^ mix64_int(blk * 0x2545F4914F6CDD1D + ctr)
        ctr += 1
        chosen.add(mix64_int(r) % k)
    return np.array(sorted(chosen), dtype=np.uint8)
