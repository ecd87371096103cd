"""Generate tests/golden/icrc_golden.npz — committed fixtures for the ICRC path.

Inputs: the three known-answer packets from the reference's own tests (tests/golden_kats.py)
plus packets built with the oracle's PacketWriter restatement over every opcode, PMTU
256..4096, pad counts 0..3, ragged lengths and random bytes.  Expected ICRCs are computed
with Python's zlib.crc32 (CRC-32/ISO-HDLC) + the reference masking — an implementation
independent of the C oracle — and bit-flip negatives record the expected verify result.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle  # noqa: E402
from golden_kats import KATS  # noqa: E402

MASK = (1, 8, 10, 11, 26, 27, 32)


def zlib_icrc(p: bytes) -> int:
    h = bytearray(p[:40])
    for o in MASK:
        h[o] = 0xFF
    return zlib.crc32(b"\xff" * 8 + bytes(h) + p[40: len(p) - 4])


def main():
    rng = np.random.default_rng(20250307)
    pkts, kinds = [], []
    for p, want in KATS:
        assert zlib_icrc(p) == want
        pkts.append(p)
        kinds.append("kat")
    opcodes = [0x06, 0x07, 0x08, 0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x0E, 0x0F, 0x10, 0x11]
    for i in range(64):
        op = opcodes[i % len(opcodes)]
        pmtu = [256, 512, 1024, 2048, 4096][i % 5]
        plen = pmtu if i % 3 else int(rng.integers(1, pmtu + 1))
        if op in (0x0C, 0x11):
            plen = int(rng.integers(0, 4))
        payload = rng.integers(0, 256, max(plen, 1), dtype=np.uint8)
        m = oracle.RdmaMsg()
        m.kind = 1 if op == 0x11 else 0
        m.opcode = op
        m.tran_type = int(rng.integers(0, 7))
        m.solicited = int(rng.integers(0, 2))
        m.ack_req = int(rng.integers(0, 2))
        m.pkey = int(rng.integers(0, 1 << 16))
        m.dqpn = int(rng.integers(0, 1 << 24))
        m.psn = int(rng.integers(0, 1 << 24))
        m.msn = int(rng.integers(0, 1 << 24))
        m.aeth_code = int(rng.integers(0, 4))
        m.aeth_value = int(rng.integers(0, 32))
        m.reth_va = int(rng.integers(0, 1 << 63))
        m.reth_rkey = int(rng.integers(0, 1 << 32))
        m.reth_len = int(rng.integers(0, 1 << 32))
        m.has_imm = 1
        m.imm = int(rng.integers(0, 1 << 32))
        m.has_secondary_reth = 1
        m.sec_va = int(rng.integers(0, 1 << 63))
        m.sec_rkey = int(rng.integers(0, 1 << 32))
        m.sec_len = int(rng.integers(0, 1 << 32))
        m.payload = payload.ctypes.data
        m.payload_len = plen
        src = int(rng.integers(0, 1 << 32))
        dst = int(rng.integers(0, 1 << 32))
        rc, p = oracle.packet_write(m, src, 4791, dst, 4791, int(rng.integers(0, 1 << 16)))
        assert rc == 0
        pkts.append(p.tobytes())
        kinds.append(f"op{op:02x}")
    for L in list(range(44, 52)) + [63, 64, 65, 127, 128, 129, 255, 257, 1083, 4155, 4157, 9001]:
        p = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        pkts.append(p)
        kinds.append("raw")
    icrc = np.array([zlib_icrc(p) for p in pkts], dtype=np.uint32)
    # negatives: trailer = ICRC, then flip one bit (outside masked bytes) in every other packet
    verify_pkts, verify_ok = [], []
    for i, p in enumerate(pkts):
        b = bytearray(p)
        b[-4:] = int(icrc[i]).to_bytes(4, "little")
        if i % 2:
            pos = int(rng.integers(0, len(b) - 4))
            while pos in MASK:
                pos = int(rng.integers(0, len(b) - 4))
            b[pos] ^= 1 << int(rng.integers(0, 8))
        verify_pkts.append(bytes(b))
        verify_ok.append(0 if i % 2 else 1)
    lens = np.array([len(p) for p in pkts], dtype=np.uint32)
    off = np.zeros(lens.size, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    np.savez_compressed(
        os.path.join(HERE, "icrc_golden.npz"),
        buf=np.frombuffer(b"".join(pkts), np.uint8), off=off, lens=lens, icrc=icrc,
        verify_buf=np.frombuffer(b"".join(verify_pkts), np.uint8),
        verify_ok=np.array(verify_ok, np.uint8), kinds=np.array(kinds))
    print(f"wrote {lens.size} packets, {int(lens.sum())} bytes")


if __name__ == "__main__":
    main()
