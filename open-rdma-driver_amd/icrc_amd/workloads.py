"""Synthetic packet streams for the BASELINE.json configurations.

Each builder returns host-side descriptors: a header-template table (n x 64 bytes, built by
patching one PacketWriter header — icrc_packet_headers — field by field with the setters'
semantics, packet.rs:100-153, 185-200, 458-515) plus icrc_synth_desc records that the
device synthesiser (icrc_synth_device) expands into full packets in HBM:

    header ‖ payload (splitmix64 stream) ‖ zero pad ‖ zero ICRC slot

Configurations
    C1  write_middle_stream(n=1 Mi, pmtu=4096): 4156-B RDMA WRITE_MIDDLE packets of one QP
    C2  mixed_mtu_stream(n): payload class in {256, 1024, 4096}, P(k) ~ k^-1.5, ~10 % ragged
        WRITE_LAST packets of U[1, k] bytes (pad 1..3)
    C3  write_message(16 MiB, 4096): one WRITE segmented like Write::handle
        (queues/send/operations/write.rs:31-96, common.rs:152-176)
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import RdmaMsg, SYNTH_DESC_DTYPE, packet_headers

OP_WRITE_FIRST = 0x06
OP_WRITE_MIDDLE = 0x07
OP_WRITE_LAST = 0x08
OP_WRITE_ONLY = 0x0A

SRC_IP = "192.168.0.2"  # queues/send/operations/common.rs:124 (hard-coded for the ICRC)
DST_IP = "192.168.0.3"
PORT = 4791


@dataclass
class Workload:
    name: str
    hdr: np.ndarray      # (n_hdr, 64) uint8 header templates
    desc: np.ndarray     # (n,) SYNTH_DESC_DTYPE
    off: np.ndarray      # (n,) uint64 packet offsets
    lens: np.ndarray     # (n,) uint32 packet lengths L (incl. ICRC)
    total_bytes: int     # buffer size needed
    stride: int = 0      # uniform stride (0 = ragged)

    @property
    def n(self) -> int:
        return int(self.lens.size)

    @property
    def payload_bytes(self) -> int:
        return int(self.desc["payload_len"].sum())


def synthesize(engine, w: "Workload", d_buf=None, stream: int = 0, pad: int = 0):
    """Expand workload `w` into packets in HBM with the device synthesiser (icrc_synth_device).
    Returns the torch uint8 buffer.  The descriptor/header tensors are kept alive until the
    stream has executed the kernel (the engine borrows device pointers until then)."""
    import torch

    if d_buf is None:
        d_buf = torch.zeros(w.total_bytes + pad, dtype=torch.uint8, device="cuda")
    d_desc = torch.from_numpy(np.ascontiguousarray(w.desc).view(np.uint8)).cuda()
    d_hdr = torch.from_numpy(np.ascontiguousarray(w.hdr)).cuda()
    engine.synth(d_buf.data_ptr(), d_desc.data_ptr(), d_hdr.data_ptr(), w.n, stream=stream)
    torch.cuda.synchronize()
    del d_desc, d_hdr
    return d_buf


def subset(w: "Workload", lo: int, hi: int) -> "Workload":
    """Packets [lo, hi) of `w` as a workload of their own, offsets rebased to the first one:
    the bytes synthesised are exactly those packets' bytes in `w` (strong-scaling shards)."""
    if not 0 <= lo <= hi <= w.n:
        raise ValueError("bad packet range")
    if lo == hi:
        return Workload(w.name, w.hdr[:0].copy(), w.desc[:0].copy(), w.off[:0].copy(), w.lens[:0].copy(), 0, w.stride)
    base = np.uint64(w.off[lo])
    desc = w.desc[lo:hi].copy()
    desc["offset"] -= base
    desc["hdr_index"] = np.arange(hi - lo, dtype=np.uint32)
    off = w.off[lo:hi] - base
    end = int(off[-1]) + int(w.lens[hi - 1])
    total = max(end, int(off[-1]) + (w.stride or 0)) if w.stride else (end + 3) // 4 * 4
    return Workload(f"{w.name}[{lo}:{hi}]", w.hdr[w.desc["hdr_index"][lo:hi]].copy(), desc, off,
                    w.lens[lo:hi].copy(), total, w.stride)


def _pad_cnt(n):
    return (4 - (n % 4)) % 4


def _template(opcode: int, payload_len: int, *, dqpn: int, msn: int, rkey: int,
              reth_len: int, ack_req: int = 0) -> tuple[np.ndarray, int]:
    m = RdmaMsg()
    m.kind = 0
    m.opcode = opcode
    m.tran_type = 0
    m.ack_req = ack_req
    m.pkey = msn
    m.dqpn = dqpn
    m.reth_rkey = rkey
    m.reth_len = reth_len & 0xFFFFFFFF
    m.payload_len = payload_len
    hdr, total = packet_headers(m, SRC_IP, PORT, DST_IP, PORT, 1)
    return hdr, total


def _patch_bth_reth(hdr: np.ndarray, opcode, payload_len, psn, ack_req, va) -> None:
    """Vectorised BTH/RETH/IPv4/UDP field writes for 56-byte BTH+RETH headers (all rows
    start from one PacketWriter template, so untouched bytes keep its values)."""
    payload_len = payload_len.astype(np.uint64)
    L = (28 + 28 + payload_len + _pad_cnt(payload_len) + 4).astype(np.uint64)
    hdr[:, 2] = (L >> 8) & 0xFF                      # Ipv4Header::set_total_length
    hdr[:, 3] = L & 0xFF
    udp = L - 20
    hdr[:, 24] = (udp >> 8) & 0xFF                   # UdpHeader::set_length
    hdr[:, 25] = udp & 0xFF
    hdr[:, 28] = (hdr[:, 28] & 0xE0) | (opcode & 0x1F)            # set_opcode_and_type (RC)
    hdr[:, 29] = (hdr[:, 29] & 0x9F) | (_pad_cnt(payload_len) << 5).astype(np.uint8)  # set_pad_cnt
    hdr[:, 36] = np.where(ack_req != 0, hdr[:, 36] | 0x80, hdr[:, 36] & 0x7F)   # set_ack_req
    psn = psn.astype(np.uint64) & 0xFFFFFF                                      # set_psn
    hdr[:, 37] = (psn >> 16) & 0xFF
    hdr[:, 38] = (psn >> 8) & 0xFF
    hdr[:, 39] = psn & 0xFF
    va = va.astype(np.uint64)
    for i in range(8):                                                          # RETH::set_va
        hdr[:, 40 + i] = (va >> np.uint64(56 - 8 * i)) & np.uint64(0xFF)


def _finish(name, hdr, payload_len, lens, payload_key, payload_pos, stride=0, align=4):
    n = lens.size
    if stride:
        off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
        total = int(n * stride)
    else:
        slots = (lens.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
        off = np.zeros(n, dtype=np.uint64)
        if n > 1:
            off[1:] = np.cumsum(slots[:-1])
        total = int(off[-1] + slots[-1]) if n else 0
    desc = np.zeros(n, dtype=SYNTH_DESC_DTYPE)
    desc["offset"] = off
    desc["payload_key"] = np.uint64(payload_key)
    desc["payload_pos"] = payload_pos
    desc["hdr_len"] = 56
    desc["payload_len"] = payload_len
    desc["total_len"] = lens
    desc["hdr_index"] = np.arange(n, dtype=np.uint32)
    return Workload(name, hdr, desc, off, lens.astype(np.uint32), total, stride)


def write_middle_stream(n: int, pmtu: int = 4096, *, stride: int | None = None,
                        remote_va: int = 0x7F7E8FC00000, dqpn: int = 2, psn0: int = 0,
                        msn: int = 0, rkey: int = 0x2000003, payload_key: int = 0x5EED5EED,
                        reth_len: int | None = None) -> Workload:
    """C1: n WRITE_MIDDLE packets of one QP; packet p carries message bytes [p*pmtu, +pmtu),
    psn = psn0 + p, RETH va = remote_va + p*pmtu (== oracle_synth_middle_stream)."""
    if reth_len is None:
        reth_len = (n * pmtu) & 0xFFFFFFFF
    t, L = _template(OP_WRITE_MIDDLE, pmtu, dqpn=dqpn, msn=msn, rkey=rkey, reth_len=reth_len)
    hdr = np.zeros((n, 64), dtype=np.uint8)
    hdr[:, : t.size] = t
    p = np.arange(n, dtype=np.uint64)
    _patch_bth_reth(hdr, np.full(n, OP_WRITE_MIDDLE, np.uint8), np.full(n, pmtu, np.uint64),
                    np.uint64(psn0) + p, np.zeros(n, np.uint8), np.uint64(remote_va) + p * np.uint64(pmtu))
    lens = np.full(n, L, dtype=np.uint32)
    return _finish("C1-write-middle", hdr, np.full(n, pmtu, np.uint32), lens, payload_key,
                   p * np.uint64(pmtu), stride=stride or L)


def mixed_mtu_stream(n: int, *, seed: int = 1234, ragged_frac: float = 0.10,
                     classes=(256, 1024, 4096), alpha: float = 1.5, dqpn: int = 3,
                     remote_va: int = 0x7F0000000000, rkey: int = 0x2000004,
                     payload_key: int = 0xC0FFEE) -> Workload:
    """C2: power-law mixed MTU with ragged LAST packets; packed 4-aligned, per-packet
    (offset, len) arrays."""
    rng = np.random.default_rng(seed)
    cls = np.asarray(classes, dtype=np.int64)
    w = cls.astype(np.float64) ** (-alpha)
    k = cls[rng.choice(cls.size, size=n, p=w / w.sum())]
    ragged = rng.random(n) < ragged_frac
    plen = np.where(ragged, rng.integers(1, k + 1), k).astype(np.uint64)
    opcode = np.where(ragged, OP_WRITE_LAST, OP_WRITE_MIDDLE).astype(np.uint8)
    t, _ = _template(OP_WRITE_MIDDLE, 4096, dqpn=dqpn, msn=0, rkey=rkey, reth_len=0)
    hdr = np.zeros((n, 64), dtype=np.uint8)
    hdr[:, : t.size] = t
    pos = np.zeros(n, dtype=np.uint64)
    if n > 1:
        pos[1:] = np.cumsum(plen[:-1])
    _patch_bth_reth(hdr, opcode, plen, np.arange(n, dtype=np.uint64), ragged.astype(np.uint8),
                    np.uint64(remote_va) + pos)
    lens = (28 + 28 + plen + _pad_cnt(plen) + 4).astype(np.uint32)
    return _finish("C2-mixed-mtu", hdr, plen.astype(np.uint32), lens, payload_key, pos)


def segments(va: int, length: int, pmtu: int):
    """generate_segments_from_request (queues/send/operations/common.rs:152-176)."""
    segs = []
    first = min(length, pmtu - ((va & 0xFFFFFFFF) % pmtu))
    segs.append((va, first))
    va += first
    rem = length - first
    while rem > 0:
        ln = min(rem, pmtu)
        segs.append((va, ln))
        va += ln
        rem -= ln
    return segs


def write_message(total_len: int = 16 << 20, pmtu: int = 4096, *, local_va: int = 0x7F7E8EE00000,
                  remote_va: int = 0x7F7E8FC00000, dqpn: int = 2, psn0: int = 0, msn: int = 0,
                  rkey: int = 0x2000003, payload_key: int = 0xABCDEF) -> Workload:
    """C3: one RDMA WRITE segmented and packetised like Write::handle (write.rs:31-96):
    FIRST/MIDDLE.../LAST (or ONLY), ack_req on LAST/ONLY, psn +1 per packet, RETH va
    advancing, RETH len = whole message length on every packet (packet.rs:427-437)."""
    segs = segments(local_va, total_len, pmtu)
    n = len(segs)
    plen = np.array([s[1] for s in segs], dtype=np.uint64)
    if n == 1:
        opcode = np.array([OP_WRITE_ONLY], np.uint8)
        ack = np.array([1], np.uint8)
    else:
        opcode = np.full(n, OP_WRITE_MIDDLE, np.uint8)
        opcode[0], opcode[-1] = OP_WRITE_FIRST, OP_WRITE_LAST
        ack = np.zeros(n, np.uint8)
        ack[-1] = 1
    pos = np.zeros(n, dtype=np.uint64)
    if n > 1:
        pos[1:] = np.cumsum(plen[:-1])
    t, _ = _template(OP_WRITE_MIDDLE, pmtu, dqpn=dqpn, msn=msn, rkey=rkey, reth_len=total_len)
    hdr = np.zeros((n, 64), dtype=np.uint8)
    hdr[:, : t.size] = t
    _patch_bth_reth(hdr, opcode, plen, np.uint64(psn0) + np.arange(n, dtype=np.uint64), ack,
                    np.uint64(remote_va) + pos)
    lens = (28 + 28 + plen + _pad_cnt(plen) + 4).astype(np.uint32)
    return _finish("C3-write-16MiB", hdr, plen.astype(np.uint32), lens, payload_key, pos)
