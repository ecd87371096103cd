"""CPU suite: the oracle against the reference's own known-answer vectors and zlib.

Pins oracle/icrc_oracle.c (restatement of packet_processor.rs:268-353 + the callers'
packet synthesis) before it is trusted as the parity checker.
"""
import zlib

import numpy as np
import pytest

import oracle
from golden_kats import IPV4_HEADERS, KAT1, KAT1_ICRC, KAT2, KAT2_ICRC, KAT3, KAT3_ICRC, \
    KAT3_UDP_PAYLOAD, KATS, SEGMENT_CASE

MASK_OFFS = (1, 8, 10, 11, 26, 27, 32)


def zlib_icrc(pkt: bytes) -> int:
    """Independent restatement with Python's zlib (CRC-32/ISO-HDLC)."""
    h = bytearray(pkt[:40])
    for o in MASK_OFFS:
        h[o] = 0xFF
    return zlib.crc32(b"\xff" * 8 + bytes(h) + pkt[40: len(pkt) - 4])


def test_crc32_check_value():
    assert oracle.crc32(b"123456789") == 0xCBF43926


@pytest.mark.parametrize("pkt,want", KATS)
def test_reference_kats(pkt, want):
    assert oracle.compute_icrc(pkt) == want
    assert zlib_icrc(pkt) == want
    assert oracle.fast_compute_icrc(pkt) == want


def test_kat_trailers_are_le():
    assert KAT1[-4:] == KAT1_ICRC.to_bytes(4, "little")
    assert KAT3[-4:] == KAT3_ICRC.to_bytes(4, "little")


def test_is_icrc_valid_semantics():
    pkt = np.frombuffer(KAT1, np.uint8).copy()
    assert oracle.is_icrc_valid(pkt)
    assert not pkt[-4:].any()                 # zeroed in place (packet_processor.rs:350)
    assert not oracle.is_icrc_valid(pkt)      # trailer now zero -> mismatch
    pkt2 = np.frombuffer(KAT2, np.uint8).copy()
    pkt2[-4:] = np.frombuffer(KAT2_ICRC.to_bytes(4, "little"), np.uint8)
    assert oracle.is_icrc_valid(pkt2)


def test_masked_bytes_do_not_change_icrc():
    base = np.frombuffer(KAT1, np.uint8).copy()
    want = oracle.compute_icrc(base)
    for o in MASK_OFFS:
        p = base.copy()
        p[o] ^= 0x5A
        assert oracle.compute_icrc(p) == want
    for o in (0, 2, 9, 12, 28, 31, 33, 40, len(base) - 5):
        p = base.copy()
        p[o] ^= 0x01
        assert oracle.compute_icrc(p) != want
    p = base.copy()
    p[-4:] = 0x77                                 # the ICRC slot is ignored
    assert oracle.compute_icrc(p) == want


def test_short_buffers_are_errors():
    for n in (0, 1, 4, 43):
        with pytest.raises(ValueError):
            oracle.compute_icrc(np.zeros(n, np.uint8))
    assert oracle.compute_icrc(np.zeros(44, np.uint8)) == zlib_icrc(bytes(44))


def test_generate_ack_kat3():
    """net/util.rs:225-239 expected UDP payload, reproduced from generate_ack's fields."""
    pkt, udp = oracle.generate_ack(0, 2, 0)
    assert udp.tobytes() == KAT3_UDP_PAYLOAD
    assert pkt.tobytes() == KAT3


def test_segments_reference_case():
    va, length, pmtu, want = SEGMENT_CASE
    assert oracle.generate_segments(va, length, pmtu) == want


def test_segments_properties():
    rng = np.random.default_rng(0)
    for _ in range(200):
        va = int(rng.integers(0, 1 << 47))
        length = int(rng.integers(0, 1 << 20))
        pmtu = int(rng.choice([256, 512, 1024, 2048, 4096]))
        segs = oracle.generate_segments(va, length, pmtu)
        assert sum(s[1] for s in segs) == length
        assert segs[0][0] == va
        for (a, la), (b, _) in zip(segs, segs[1:]):
            assert b == a + la
            assert (b & 0xFFFFFFFF) % pmtu == 0


@pytest.mark.parametrize("hdr,want", IPV4_HEADERS)
def test_ipv4_checksum(hdr, want):
    assert oracle.ipv4_checksum(hdr) == want


def test_fast_core_equals_table_core():
    rng = np.random.default_rng(3)
    for n in list(range(0, 300)) + [4096, 4152, 5000, 65535, 100000]:
        d = rng.integers(0, 256, n, dtype=np.uint8)
        c0 = int(rng.integers(0, 1 << 32))
        assert oracle.fast_crc32(d, c0) == oracle.crc32(d, c0) == zlib.crc32(d.tobytes(), c0)


def test_packet_writer_zlib_crosscheck():
    """PacketWriter restatement: every opcode, pad 0..3; ICRC cross-checked with zlib and
    header fields with the setters' semantics (packet.rs:100-243, 458-515)."""
    rng = np.random.default_rng(4)
    for opcode, hl in ((0x06, 28), (0x07, 28), (0x08, 28), (0x0A, 28), (0x0D, 28), (0x0E, 28),
                       (0x0F, 28), (0x10, 28), (0x09, 32), (0x0B, 32), (0x0C, 44), (0x11, 16)):
        for plen in (0, 1, 2, 3, 4, 5, 1024, 4093):
            payload = rng.integers(0, 256, max(plen, 1), dtype=np.uint8)
            m = oracle.RdmaMsg()
            m.kind = 1 if opcode == 0x11 else 0
            m.opcode = opcode
            m.tran_type = 0
            m.ack_req = 1
            m.solicited = 1
            m.pkey = 0xBEEF
            m.dqpn = 0x123456
            m.psn = 0xFEDCBA
            m.msn = 0x0A0B0C
            m.aeth_value = 0x1F
            m.reth_va = 0x7F7E91000000
            m.reth_rkey = 0x01709A33
            m.reth_len = 0x80
            m.has_imm = 1
            m.imm = 0x01020304
            m.has_secondary_reth = 1
            m.payload = payload.ctypes.data
            m.payload_len = plen
            rc, pkt = oracle.packet_write(m, 0xC0A80002, 4791, 0xC0A80003, 4791, 1)
            assert rc == 0
            pad = (4 - plen % 4) % 4
            L = 28 + hl + plen + pad + 4
            assert pkt.size == L
            assert int.from_bytes(pkt[2:4].tobytes(), "big") == L
            assert int.from_bytes(pkt[24:26].tobytes(), "big") == L - 20
            assert pkt[28] == opcode
            assert (pkt[29] >> 5) & 3 == pad and pkt[29] & 0x80
            assert pkt[32] == 0 and int.from_bytes(pkt[33:36].tobytes(), "big") == 0x123456
            assert pkt[36] & 0x80 and int.from_bytes(pkt[37:40].tobytes(), "big") == 0xFEDCBA
            assert pkt[28 + hl: 28 + hl + plen].tobytes() == payload[:plen].tobytes()
            assert not pkt[28 + hl + plen: L - 4].any()
            assert int.from_bytes(pkt[L - 4:].tobytes(), "little") == zlib_icrc(pkt.tobytes())


def test_packet_writer_errors():
    m = oracle.RdmaMsg()
    m.kind = 1
    m.opcode = 0x07  # General opcode with Acknowledge metadata
    assert oracle.packet_write(m, 1, 1, 2, 2, 1)[0] == oracle.INVALID_METADATA
    m.kind = 0
    m.opcode = 0x1F
    assert oracle.packet_write(m, 1, 1, 2, 2, 1)[0] == oracle.INVALID_OPCODE
    m.opcode = 0x07
    big = np.zeros(70000, np.uint8)
    m.payload = big.ctypes.data
    m.payload_len = 65535
    assert oracle.packet_write(m, 1, 1, 2, 2, 1, buf_len=80000)[0] == oracle.LENGTH_TOO_LONG
    m.payload_len = 100
    assert oracle.packet_write(m, 1, 1, 2, 2, 1, buf_len=100)[0] == oracle.BUFFER_NOT_LARGE


def test_synth_write_stream_shape():
    buf, off, lens = oracle.synth_write(256 << 10, 4096, local_va=0x7F0000000000,
                                        remote_va=0x7F7E8FC00000, rkey=3, dqpn=2, psn0=5, msn=9,
                                        dst_ip=0xC0A80003, payload_key=1)
    assert lens.size == 64 and set(lens.tolist()) == {4156}
    ops = [int(buf[int(o) + 28]) for o in off]
    assert ops[0] == 0x06 and ops[-1] == 0x08 and set(ops[1:-1]) == {0x07}
    psns = [int.from_bytes(buf[int(o) + 37: int(o) + 40].tobytes(), "big") for o in off]
    assert psns == list(range(5, 69))
    for o, L in zip(off, lens):
        p = buf[int(o): int(o) + int(L)]
        assert int.from_bytes(p[-4:].tobytes(), "little") == zlib_icrc(p.tobytes())
