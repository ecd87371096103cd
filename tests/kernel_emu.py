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


def _bswap32(x: int) -> int:
    return int.from_bytes((x & 0xFFFFFFFF).to_bytes(4, "little"), "big")


def _bswap16(x: int) -> int:
    return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)


def packetizer_header_words(m, s: int) -> tuple:
    """icrc_packetize_kernel's plan_packet + header_lanes for packet s of message m (a
    WRITE_MSG_DTYPE record): returns (14, 15 or 18 LE header words, payload len, wire length L)."""
    kind, flags = int(m["kind"]), int(m["flags"])
    if kind == 2:  # READ REQUEST: one packet, no payload, a secondary RETH (read.rs:57-74)
        start, ln, hw = 0, 0, 18
    else:
        total, pmtu = int(m["total_len"]), int(m["pmtu"])
        seg_va = int(m["remote_va"]) if flags & 0x02 else int(m["local_va"])  # ICRC_WRITE_RUST_DRIVER
        first = min(total, pmtu - (seg_va & 0xFFFFFFFF) % pmtu)
        if s == 0:
            start, ln = 0, first
        else:
            start = first + (s - 1) * pmtu
            ln = min(pmtu, total - start)
        hw = 14
    pad = (4 - (ln & 3)) & 3
    L = 4 * hw + ln + pad + 4
    n = int(m["npackets"])
    only, last = n == 1, s + 1 == n
    rlen = int(m["reth_len"])
    if kind == 2:
        op, ack = 0x0C, 1 if flags & 0x08 else 0
    elif not flags & 0x02:  # emulator: Write::handle / ReadResponse::handle
        ONLY, FIRST, MIDDLE, LAST = (0x0A, 0x06, 0x07, 0x08) if kind == 0 else (0x10, 0x0D, 0x0E, 0x0F)
        op = ONLY if only else (FIRST if s == 0 else (LAST if last else MIDDLE))
        ack = 1 if (only or last) else 0
    else:  # send_opcode, ICRC_WRITE_RUST_DRIVER
        df, dl = not flags & 0x20, not flags & 0x40
        imm = kind == 0 and bool(flags & 0x80)
        ONLY, FIRST, MIDDLE = (0x0A, 0x06, 0x07) if kind == 0 else (0x10, 0x0D, 0x0E)
        LAST = 0x0F if kind == 1 else (0x09 if imm else 0x08)
        if only:
            op = (0x0B if imm else ONLY) if (df and dl) else (FIRST if df else LAST)
        elif s == 0:
            op = FIRST if df else MIDDLE
        elif not last:
            op = MIDDLE
        else:
            op = LAST if dl else MIDDLE
        ack = 1 if flags & 0x08 else 0
        rlen = rlen if op == FIRST else ln
        if op in (0x09, 0x0B):
            hw = 15
            L = 4 * hw + ln + pad + 4
    sol = 0x80 if flags & 0x04 else 0
    psn = (int(m["psn"]) + s) & 0xFFFFFF
    va = (int(m["remote_va"]) + start) & 0xFFFFFFFFFFFFFFFF
    w = [0] * hw
    w[0] = 0x45 | (((L >> 8) & 0xFF) << 16) | ((L & 0xFF) << 24)
    w[1] = _bswap16(int(m["ip_id"]))
    w[2] = 0x1140
    w[3] = _bswap32(int(m["src_ip"]))
    w[4] = _bswap32(int(m["dst_ip"]))
    w[5] = _bswap16(4791) | (_bswap16(4791) << 16)
    w[6] = _bswap16(L - 20)
    w[7] = (((int(m["tran_type"]) << 5) & 0xFF) | op) | ((sol | (pad << 5)) << 8) | (_bswap16(int(m["msn"])) << 16)
    w[8] = _bswap32(int(m["dqpn"]) & 0xFFFFFF)
    w[9] = _bswap32(psn) | (ack << 7)
    w[10] = _bswap32(va >> 32)
    w[11] = _bswap32(va & 0xFFFFFFFF)
    w[12] = _bswap32(int(m["rkey"]))
    w[13] = _bswap32(rlen)
    if hw == 15:
        w[14] = _bswap32(int(m["imm"]))
    if hw == 18:
        lva = int(m["local_va"])
        w[14] = _bswap32(lva >> 32)
        w[15] = _bswap32(lva & 0xFFFFFFFF)
        w[16] = _bswap32(int(m["lkey"]))
        w[17] = _bswap32(int(m["total_len"]))
    if flags & 0x01:
        src, dst = int(m["src_ip"]), int(m["dst_ip"])
        sm = 0x4500 + L + int(m["ip_id"]) + 0x4011 + (src >> 16) + (src & 0xFFFF) + (dst >> 16) + (dst & 0xFFFF)
        sm = (sm & 0xFFFF) + (sm >> 16)
        sm = (sm & 0xFFFF) + (sm >> 16)
        w[2] |= _bswap16(~sm & 0xFFFF) << 16
    return tuple(w), ln, L


def head_mask(k: np.ndarray) -> np.ndarray:
    """icrc_device.h head_mask: OR-mask of stream word k (FF prefix, masked header bytes)."""
    out = np.zeros(k.size, dtype=np.uint32)
    for i, kk in enumerate(k):
        if 0 <= kk < 16:
            nib = (0x00000010C000D02F >> (4 * int(kk))) & 15
            out[i] = sum(0xFF << (8 * t) for t in range(4) if nib >> t & 1)
    return out


def icrc_rows_aligned(img: np.ndarray, pkt: np.ndarray, rows: int = 17) -> int:
    """The packetizer's ring slot (icrc_packetize_kernel process): the packet END-aligned in
    `rows` rows of 64 words with leading zero rows, head masks only on the two rows holding
    stream words 0..9, every row stepped (a zero accumulator stays zero)."""
    L = pkt.size
    assert L % 4 == 0
    N = 1 + (L - 4) // 4
    k0 = N - 64 * rows
    assert k0 <= 0
    lane = np.arange(64, dtype=np.int64)
    words = np.frombuffer(pkt[: L - 4].tobytes(), "<u4")
    j0 = (-k0) >> 6
    acc = np.zeros(64, dtype=np.uint32)
    for j in range(rows):
        k = k0 + lane + 64 * j          # stream word; packet word k - 1
        w = np.array([words[x - 1] if 1 <= x <= words.size else 0 for x in k], dtype=np.uint32)
        u = w | (head_mask(k) if j in (j0, j0 + 1) else np.uint32(0))
        acc = u if j == 0 else (mul_m64(img, acc) ^ u)
    s = np.bitwise_xor.reduce(final_mul(img, acc))
    return int(~np.uint32(s) & 0xFFFFFFFF)


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


# ---- the oct kernel's per-packet path (group_slow_packet, icrc_device.h): W lanes per packet ----
def _step_lanes(img, s, lanes):
    lo0 = (lanes & 31) * 4
    lo1 = lo0 + 128
    a0 = ((s << 8) & 0xFF00) | lo0
    a1 = (s & 0xFF00) | lo1
    a2 = ((s >> 8) & 0xFF00) | (lo0 + 65536)
    a3 = ((s >> 16) & 0xFF00) | (lo1 + 65536)
    return _lds(img, a0) ^ _lds(img, a1) ^ _lds(img, a2) ^ _lds(img, a3)


def icrc_group(img: np.ndarray, pkt: np.ndarray, group: int = 0, lead: int = 0, W: int = 8) -> int:
    """One packet on lanes W*group .. W*group+W-1 of the oct kernel (W = 8), on its table image: end-aligned rows of W stream words, `lead` extra leading zero
    rows (a shorter packet of a set runs behind the set's longest one), acc <- M^W(acc) ^ u,
    then XOR_c M^(W-c)(acc_c)."""
    Ld = pkt.size - 4
    T = 4 + Ld
    z = (4 - (T & 3)) & 3
    N = (T + z) >> 2
    R = (N + W - 1) // W
    k0 = N - W * R
    lanes = np.arange(W, dtype=np.uint32) + W * group
    col = np.arange(W, dtype=np.int64)
    acc = np.zeros(W, dtype=np.uint32)
    for r in range(-lead, R):
        u = stream_words(pkt, z, k0 + W * r + col) if r >= 0 else np.zeros(W, np.uint32)
        acc = _step_lanes(img, acc, lanes) ^ u
    fin = KFINAL + lanes * 4
    f = np.zeros(W, dtype=np.uint32)
    for n in range(8):
        f ^= _lds(img, fin + n * 4096 + (((acc >> (4 * n)) & 15) << 8))
    return int(~np.uint32(np.bitwise_xor.reduce(f)) & 0xFFFFFFFF)


# ---- oct kernel (icrc_oct.hip): eight packets per wavefront in chained 10-row frames -----------
def icrc_oct_set(img: np.ndarray, pkts, K: int = 10) -> list:
    """One set of up to eight 4-aligned packets (L % 4 == 0) the way icrc_oct.hip steps it: lane
    8g + c carries packet g; stream word 8 r + c - z in row r (z = -N mod 8 front padding, so rows
    are aligned to both ends of the packet); the header masks of rows 0..2 come from a lane table
    (lane k holds head_mask(k)) read at (kf + 8 j) & 63 — negative k wraps to lanes 57..63, which
    hold 0; the set runs ceil(Rmax / K) frames of K rows with the accumulator carried; a packet's
    lanes freeze past its own last row.  Returns the ICRCs."""
    hm_lane = head_mask(np.arange(64, dtype=np.int64))
    ng = len(pkts)
    lanes = np.arange(64, dtype=np.uint32)
    grp = lanes >> 3
    col = (lanes & 7).astype(np.int64)
    N = np.zeros(64, np.int64)
    R = np.zeros(64, np.int64)
    words = []
    for g in range(8):
        if g < ng:
            L = pkts[g].size
            assert L % 4 == 0 and L >= 44
            n = 1 + (L - 4) // 4
            words.append(np.frombuffer(pkts[g][: L - 4].tobytes(), "<u4"))
        else:
            n = 0
            words.append(np.zeros(0, np.uint32))
        N[grp == g] = n
        R[grp == g] = (n + 7) // 8
    z = (8 - (N & 7)) & 7
    kf = col - z                               # stream word of this lane in row 0
    rmax = int(R.max())
    acc = np.zeros(64, dtype=np.uint32)
    for f in range((rmax + K - 1) // K):
        for j in range(K):
            r = K * f + j
            if r >= rmax:
                break
            k = kf + 8 * r
            u = np.zeros(64, np.uint32)
            for i in range(64):
                g = int(grp[i])
                if 1 <= k[i] <= words[g].size:
                    u[i] = words[g][k[i] - 1]
            if r < 3:
                u |= hm_lane[(k & 63).astype(np.int64)]
            nv = u if r == 0 else (_step_lanes(img, acc, lanes) ^ u)
            acc = np.where(r < R, nv, acc).astype(np.uint32)
    fin = KFINAL + lanes * 4
    fm = np.zeros(64, dtype=np.uint32)
    for n in range(8):
        fm ^= _lds(img, fin + n * 4096 + (((acc >> (4 * n)) & 15) << 8))
    return [int(~np.uint32(np.bitwise_xor.reduce(fm[8 * g: 8 * g + 8])) & 0xFFFFFFFF) for g in range(ng)]
