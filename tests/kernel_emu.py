"""kernel_emu.py — numpy emulation of the HIP kernel's lane algorithm (test helper).

Mirrors icrc_kernels.hip step by step (end-aligned word rows, per-lane Horner with the
M^64 byte tables, per-lane M^(64-l) nibble tables, XOR over lanes) on the very table image
the product uploads (icrc_table_image).  Lets the CPU suite check the algorithm and the
table layout against the oracle without a GPU.  Never used by the product.
"""
import numpy as np

KFINAL = 131072
MASK_OFFS = (1, 8, 10, 11, 26, 27, 32)


def _lds(img, addr):
    return img[np.asarray(addr, dtype=np.int64) >> 2]


def mul_m64(img, s):
    lane = np.arange(64, dtype=np.uint32)
    lo0 = (lane & 31) * 4
    lo1 = lo0 + 128
    a0 = ((s << 8) & 0xFF00) | lo0
    a1 = (s & 0xFF00) | lo1
    a2 = ((s >> 8) & 0xFF00) | (lo0 + 65536)
    a3 = ((s >> 16) & 0xFF00) | (lo1 + 65536)
    return _lds(img, a0) ^ _lds(img, a1) ^ _lds(img, a2) ^ _lds(img, a3)


def final_mul(img, acc):
    lane = np.arange(64, dtype=np.uint32)
    fin = KFINAL + lane * 4
    r = np.zeros(64, dtype=np.uint32)
    for n in range(8):
        r ^= _lds(img, fin + n * 4096 + (((acc >> (4 * n)) & 15) << 8))
    return r


def stream_words(pkt: np.ndarray, z: int, k: np.ndarray) -> np.ndarray:
    """Value of stream word k (generic path semantics, any alignment)."""
    Ld = pkt.size - 4
    out = np.zeros(k.size, dtype=np.uint32)
    for idx, kk in enumerate(k):
        if kk < 0:
            continue
        w = 0
        for t in range(4):
            j = 4 * int(kk) + t - z
            if j < 0:
                b = 0
            elif j < 4:
                b = 0xFF
            else:
                o = j - 4
                assert o < Ld
                b = 0xFF if o in MASK_OFFS else int(pkt[o])
            w |= b << (8 * t)
        out[idx] = w
    return out


def icrc(img: np.ndarray, pkt: np.ndarray) -> int:
    Ld = pkt.size - 4
    T = 4 + Ld
    z = (4 - (T & 3)) & 3
    N = (T + z) >> 2
    R = (N + 63) >> 6
    k0 = N - 64 * R
    lane = np.arange(64, dtype=np.int64)
    acc = np.zeros(64, dtype=np.uint32)
    for r in range(R):
        u = stream_words(pkt, z, k0 + 64 * r + lane)
        acc = u if r == 0 else (mul_m64(img, acc) ^ u)
    s = np.bitwise_xor.reduce(final_mul(img, acc))
    return int(~np.uint32(s) & 0xFFFFFFFF)
