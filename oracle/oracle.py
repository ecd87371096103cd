"""oracle.py — TEST INFRASTRUCTURE ONLY: ctypes loader for the CPU restatement.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker.  The product path (open-rdma-driver_amd/) never imports it.

Every wrapped function restates the reference ICRC path; see icrc_oracle.c for the
file:line each one follows (packet_processor.rs:268-353 for compute/verify).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

OK = 0
EINVAL = -22
BUFFER_NOT_LARGE = -1000
LENGTH_TOO_LONG = -1001
INVALID_METADATA = -1002
INVALID_OPCODE = -1003

OP_WRITE_FIRST = 0x06
OP_WRITE_MIDDLE = 0x07
OP_WRITE_LAST = 0x08
OP_WRITE_LAST_IMM = 0x09
OP_WRITE_ONLY = 0x0A
OP_WRITE_ONLY_IMM = 0x0B
OP_READ_REQUEST = 0x0C
OP_READ_RESP_FIRST = 0x0D
OP_READ_RESP_MIDDLE = 0x0E
OP_READ_RESP_LAST = 0x0F
OP_READ_RESP_ONLY = 0x10
OP_ACK = 0x11


class WriteDesc(ctypes.Structure):
    """oracle_write_desc (icrc_oracle.h): the ToCardWriteDescriptor fields BlueRDMALogic::send reads."""

    _fields_ = [
        ("raddr", ctypes.c_uint64), ("total_len", ctypes.c_uint32), ("sge_len", ctypes.c_uint32),
        ("pmtu", ctypes.c_uint32), ("psn", ctypes.c_uint32), ("imm", ctypes.c_uint32),
        ("is_resp", ctypes.c_uint8), ("is_first", ctypes.c_uint8), ("is_last", ctypes.c_uint8),
        ("has_imm", ctypes.c_uint8),
    ]


class LogicPkt(ctypes.Structure):
    """oracle_logic_pkt (icrc_oracle.h): one RdmaMessage BlueRDMALogic::send emits."""

    _fields_ = [
        ("reth_va", ctypes.c_uint64), ("psn", ctypes.c_uint32), ("reth_len", ctypes.c_uint32),
        ("imm", ctypes.c_uint32), ("payload_off", ctypes.c_uint32), ("payload_len", ctypes.c_uint32),
        ("opcode", ctypes.c_uint8), ("has_imm", ctypes.c_uint8), ("_pad", ctypes.c_uint8 * 2),
    ]


class RdmaMsg(ctypes.Structure):
    """Flattened RdmaMessage (types.rs); layout == oracle_rdma_msg in icrc_oracle.h."""

    _fields_ = [
        ("kind", ctypes.c_uint8),
        ("opcode", ctypes.c_uint8),
        ("tran_type", ctypes.c_uint8),
        ("solicited", ctypes.c_uint8),
        ("ack_req", ctypes.c_uint8),
        ("aeth_code", ctypes.c_uint8),
        ("aeth_value", ctypes.c_uint8),
        ("has_imm", ctypes.c_uint8),
        ("has_secondary_reth", ctypes.c_uint8),
        ("_pad0", ctypes.c_uint8 * 3),
        ("pkey", ctypes.c_uint16),
        ("_pad1", ctypes.c_uint16),
        ("dqpn", ctypes.c_uint32),
        ("psn", ctypes.c_uint32),
        ("msn", ctypes.c_uint32),
        ("imm", ctypes.c_uint32),
        ("reth_va", ctypes.c_uint64),
        ("reth_rkey", ctypes.c_uint32),
        ("reth_len", ctypes.c_uint32),
        ("sec_va", ctypes.c_uint64),
        ("sec_rkey", ctypes.c_uint32),
        ("sec_len", ctypes.c_uint32),
        ("payload", ctypes.c_void_p),
        ("payload_len", ctypes.c_uint64),
    ]


def build() -> str:
    """Compile the oracle library (gcc) if needed; returns its path."""
    srcs = [os.path.join(_HERE, f) for f in ("icrc_oracle.c", "icrc_fast.c", "icrc_oracle.h")]
    if not os.path.exists(_LIB_PATH) or any(
        os.path.getmtime(s) > os.path.getmtime(_LIB_PATH) for s in srcs
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.oracle_crc32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_crc32.restype = ctypes.c_uint32
        L.oracle_compute_icrc.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_compute_icrc.restype = ctypes.c_int
        L.oracle_is_icrc_valid.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
        L.oracle_is_icrc_valid.restype = ctypes.c_int
        L.oracle_compute_icrc_batch.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, u8p]
        L.oracle_compute_icrc_batch.restype = ctypes.c_int
        L.oracle_packet_write.argtypes = [
            u8p, ctypes.c_size_t, ctypes.POINTER(RdmaMsg), ctypes.c_uint32, ctypes.c_uint16,
            ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint16, ctypes.POINTER(ctypes.c_size_t),
        ]
        L.oracle_packet_write.restype = ctypes.c_int
        L.oracle_generate_ack.argtypes = [ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32, u8p, u8p]
        L.oracle_generate_ack.restype = ctypes.c_int
        L.oracle_generate_segments.argtypes = [
            ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u8p, u8p, ctypes.c_uint32,
        ]
        L.oracle_generate_segments.restype = ctypes.c_uint32
        L.oracle_logic_send.argtypes = [ctypes.POINTER(WriteDesc), ctypes.POINTER(LogicPkt), ctypes.c_uint32]
        L.oracle_logic_send.restype = ctypes.c_uint32
        L.oracle_ipv4_checksum.argtypes = [u8p]
        L.oracle_ipv4_checksum.restype = ctypes.c_uint16
        L.oracle_mix64.argtypes = [ctypes.c_uint64]
        L.oracle_mix64.restype = ctypes.c_uint64
        L.oracle_header_len.argtypes = [ctypes.c_uint8]
        L.oracle_header_len.restype = ctypes.c_int
        L.oracle_rx_parse.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, u8p]
        L.oracle_rx_parse.restype = ctypes.c_int
        L.oracle_rx_parse_batch.argtypes = [u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_int, u8p]
        L.oracle_rx_parse_batch.restype = ctypes.c_int
        L.oracle_synth_write.argtypes = [
            u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
            ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64,
        ]
        L.oracle_synth_write.restype = ctypes.c_int64
        L.oracle_synth_middle_stream.argtypes = [
            u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_uint64, ctypes.c_uint32,
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16,
            ctypes.c_uint32, ctypes.c_uint64,
        ]
        L.oracle_synth_middle_stream.restype = ctypes.c_int64
        L.fast_crc32.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.fast_crc32.restype = ctypes.c_uint32
        L.fast_crc32_slice16.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.fast_crc32_slice16.restype = ctypes.c_uint32
        L.fast_compute_icrc.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)]
        L.fast_compute_icrc.restype = ctypes.c_int
        L.fast_icrc_strided_timed.argtypes = [
            u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, u8p, ctypes.c_int,
        ]
        L.fast_icrc_strided_timed.restype = ctypes.c_double
        L.fast_emulator_path_timed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, u8p]
        L.fast_emulator_path_timed.restype = ctypes.c_double
        L.fast_verify_strided_timed.argtypes = [
            u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, u8p, ctypes.c_int, ctypes.c_int,
        ]
        L.fast_verify_strided_timed.restype = ctypes.c_double
        L.fast_c0_roundtrip_timed.argtypes = [
            u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
        ]
        L.fast_c0_roundtrip_timed.restype = ctypes.c_double
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _as_u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def crc32(data, crc: int = 0) -> int:
    a = _as_u8(data)
    return lib().oracle_crc32(crc, _ptr(a), a.size)


def compute_icrc(pkt) -> int:
    """compute_icrc (packet_processor.rs:275-301). Raises ValueError where the reference panics."""
    a = _as_u8(pkt)
    out = ctypes.c_uint32()
    rc = lib().oracle_compute_icrc(_ptr(a), a.size, ctypes.byref(out))
    if rc:
        raise ValueError(f"compute_icrc: rc={rc}")
    return out.value


def is_icrc_valid(pkt: np.ndarray) -> bool:
    """is_icrc_valid (packet_processor.rs:341-353); zeroes the trailer of `pkt` in place."""
    assert isinstance(pkt, np.ndarray) and pkt.dtype == np.uint8 and pkt.flags.c_contiguous
    ok = ctypes.c_int()
    rc = lib().oracle_is_icrc_valid(_ptr(pkt), pkt.size, ctypes.byref(ok))
    if rc:
        raise ValueError(f"is_icrc_valid: rc={rc}")
    return bool(ok.value)


def compute_icrc_batch(base: np.ndarray, off: np.ndarray, lens: np.ndarray) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.zeros(off.size, dtype=np.uint32)
    rc = lib().oracle_compute_icrc_batch(_ptr(base), _ptr(off), _ptr(lens), off.size, _ptr(out))
    if rc:
        raise ValueError(f"compute_icrc_batch: rc={rc}")
    return out


def packet_write(msg: RdmaMsg, src_ip: int, src_port: int, dst_ip: int, dst_port: int,
                 ip_id: int, buf_len: int = 8192):
    """PacketWriter::write (packet_processor.rs:210-265) into a zeroed buffer.
    Returns (rc, packet bytes as np.uint8 array of length L, or None)."""
    buf = np.zeros(buf_len, dtype=np.uint8)
    n = ctypes.c_size_t()
    rc = lib().oracle_packet_write(_ptr(buf), buf_len, ctypes.byref(msg), src_ip, src_port,
                                   dst_ip, dst_port, ip_id, ctypes.byref(n))
    if rc:
        return rc, None
    return rc, buf[: n.value].copy()


def generate_ack(pkey: int, peer_qpn: int, expected_psn: int):
    pkt = np.zeros(48, dtype=np.uint8)
    udp = np.zeros(20, dtype=np.uint8)
    rc = lib().oracle_generate_ack(pkey, peer_qpn, expected_psn, _ptr(pkt), _ptr(udp))
    if rc:
        raise ValueError(f"generate_ack: rc={rc}")
    return pkt, udp


def generate_segments(va: int, length: int, pmtu: int):
    n = lib().oracle_generate_segments(va, length, pmtu, None, None, 0)
    sva = np.zeros(n, dtype=np.uint64)
    sl = np.zeros(n, dtype=np.uint32)
    lib().oracle_generate_segments(va, length, pmtu, _ptr(sva), _ptr(sl), n)
    return [(int(a), int(b)) for a, b in zip(sva, sl)]


def logic_send(*, raddr: int, total_len: int, sge_len: int, pmtu: int, psn: int, is_resp: bool = False,
               is_first: bool = True, is_last: bool = True, imm=None) -> list:
    """BlueRDMALogic::send (rust_driver/src/device/software/logic.rs:191-271) for one WRITE /
    WRITE_WITH_IMM / READ_RESP descriptor: the RdmaMessages it hands to NetSendAgent::send, as
    dicts (opcode, psn, reth_va, reth_len, imm or None, payload_off, payload_len)."""
    d = WriteDesc(raddr=raddr & 0xFFFFFFFFFFFFFFFF, total_len=total_len, sge_len=sge_len, pmtu=pmtu, psn=psn,
                  imm=0 if imm is None else imm, is_resp=int(is_resp), is_first=int(is_first),
                  is_last=int(is_last), has_imm=int(imm is not None))
    n = lib().oracle_logic_send(ctypes.byref(d), None, 0)
    out = (LogicPkt * max(n, 1))()
    lib().oracle_logic_send(ctypes.byref(d), out, n)
    return [dict(opcode=p.opcode, psn=p.psn, reth_va=p.reth_va, reth_len=p.reth_len,
                 imm=p.imm if p.has_imm else None, payload_off=p.payload_off, payload_len=p.payload_len)
            for p in out[:n]]


def ipv4_checksum(hdr) -> int:
    a = _as_u8(hdr)
    return lib().oracle_ipv4_checksum(_ptr(a))


def mix64(x: int) -> int:
    return lib().oracle_mix64(x & 0xFFFFFFFFFFFFFFFF)


def synth_write(total_len: int, pmtu: int, *, local_va: int, remote_va: int, rkey: int,
                dqpn: int, psn0: int, msn: int, dst_ip: int, payload_key: int,
                stride: int | None = None):
    """Emulator WRITE send path; returns (buffer, offsets, lens)."""
    n = len(generate_segments(local_va, total_len, pmtu))
    stride = stride or ((28 + 28 + pmtu + 4 + 3) // 4 * 4)
    buf = np.zeros(n * stride, dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint32)
    got = lib().oracle_synth_write(_ptr(buf), stride, n, _ptr(lens), local_va, remote_va,
                                   total_len, pmtu, rkey, dqpn, psn0, msn, dst_ip, payload_key)
    if got != n:
        raise ValueError(f"synth_write: rc={got}")
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    return buf, off, lens


RX_DESC_DTYPE = np.dtype([  # oracle_rx_desc (icrc_oracle.h)
    ("reth_va", "<u8"), ("sec_va", "<u8"), ("payload_offset", "<u8"), ("payload_len", "<u4"),
    ("reth_rkey", "<u4"), ("reth_len", "<u4"), ("sec_rkey", "<u4"), ("sec_len", "<u4"),
    ("imm", "<u4"), ("dqpn", "<u4"), ("psn", "<u4"), ("aeth_msn", "<u4"), ("pkey", "<u2"),
    ("opcode", "u1"), ("tran_type", "u1"), ("flags", "u1"), ("pad_cnt", "u1"),
    ("aeth_code", "u1"), ("aeth_value", "u1"), ("icrc_ok", "u1"), ("status", "u1"),
    ("_pad", "u1", (2,)),
])
assert RX_DESC_DTYPE.itemsize == 72


def rx_parse(base: np.ndarray, off, lens, zero_trailer: bool = False) -> np.ndarray:
    """is_icrc_valid + to_rdma_message(pkt[28 .. L-4)) per packet (icrc_oracle.c
    oracle_rx_parse, looped in C by oracle_rx_parse_batch); `base` is modified only when
    zero_trailer."""
    off = np.ascontiguousarray(off, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    out = np.zeros(off.size, dtype=RX_DESC_DTYPE)
    if off.size:
        rc = lib().oracle_rx_parse_batch(_ptr(base), off.ctypes.data, lens.ctypes.data, off.size,
                                         1 if zero_trailer else 0, out.ctypes.data)
        if rc != 0:
            raise ValueError(f"oracle_rx_parse_batch: {rc}")
    return out


_SEND_OPCODES = {  # (only, first, middle, last): write.rs:31-96, read_response.rs:30-95
    0: (0x0A, 0x06, 0x07, 0x08),
    1: (0x10, 0x0D, 0x0E, 0x0F),
}


def send_messages(src: np.ndarray, msgs: np.ndarray, wire_bytes: int):
    """The emulator's send step for an icrc_write_msg array (fields as in include/icrc.h):
    per message generate_segments_from_request (common.rs:152-176), per segment the Write /
    ReadResponse handler's opcode / PSN / ack_req / RETH choice and send_write_message
    (common.rs:73-132) -> generate_payload_from_msg -> PacketWriter::write with the ICRC
    trailer.  Returns (wire, pkt_len, icrc) with packets at out_offset + s * slot_stride."""
    wire = np.zeros(wire_bytes, dtype=np.uint8)
    npk = int(msgs["npackets"].sum()) if len(msgs) else 0
    lens = np.zeros(npk, dtype=np.uint32)
    icrcs = np.zeros(npk, dtype=np.uint32)
    for m in msgs:
        flags = int(m["flags"]) if "flags" in m.dtype.names else 0
        if int(m["kind"]) == 2:  # Read::handle (read.rs:33-89): one request packet, no payload
            assert int(m["npackets"]) == 1
            msg = RdmaMsg()
            msg.kind = 0
            msg.opcode = OP_READ_REQUEST
            msg.tran_type = int(m["tran_type"])
            msg.solicited = 1 if flags & 0x04 else 0
            msg.ack_req = 1 if flags & 0x08 else 0  # send_flag == IbvSendSignaled (read.rs:37)
            msg.pkey = int(m["msn"])
            msg.dqpn = int(m["dqpn"])
            msg.psn = int(m["psn"])
            msg.reth_va = int(m["remote_va"])
            msg.reth_rkey = int(m["rkey"])
            msg.reth_len = int(m["reth_len"])
            msg.has_secondary_reth = 1
            msg.sec_va = int(m["local_va"])
            msg.sec_rkey = int(m["lkey"])
            msg.sec_len = int(m["total_len"])
            msg.payload = None
            msg.payload_len = 0
            rc, pkt = packet_write(msg, int(m["src_ip"]), 4791, int(m["dst_ip"]), 4791, int(m["ip_id"]))
            if rc or pkt.size > 0xFFFF:
                raise ValueError(f"packet_write rc={rc}")
            if flags & 0x01:
                c = ipv4_checksum(pkt[:20])
                pkt[10], pkt[11] = c >> 8, c & 0xFF
            o = int(m["out_offset"])
            wire[o: o + pkt.size] = pkt
            k = int(m["first_packet"])
            lens[k], icrcs[k] = pkt.size, int(pkt[-4:].view("<u4")[0])
            continue
        if flags & 0x02:  # ICRC_WRITE_RUST_DRIVER: BlueRDMALogic::send (logic.rs:168-271)
            plan = logic_send(raddr=int(m["remote_va"]), total_len=int(m["reth_len"]), sge_len=int(m["total_len"]),
                              pmtu=int(m["pmtu"]), psn=int(m["psn"]), is_resp=int(m["kind"]) == 1,
                              is_first=not flags & 0x20, is_last=not flags & 0x40,
                              imm=int(m["imm"]) if (flags & 0x80 and int(m["kind"]) == 0) else None)
            ack_all = 1 if flags & 0x08 else 0  # ack_req: false (logic.rs:184) unless ICRC_WRITE_ACK_REQ
            plan = [(p["opcode"], ack_all, p["psn"], p["reth_va"], p["reth_len"], p["imm"], p["payload_len"])
                    for p in plan]
        else:
            segs = generate_segments(int(m["local_va"]), int(m["total_len"]), int(m["pmtu"]))
            only, first, middle, last = _SEND_OPCODES[int(m["kind"])]
            plan, pos = [], 0
            for s, (_, sl) in enumerate(segs):
                if len(segs) == 1:
                    op, ack = only, 1
                elif s == 0:
                    op, ack = first, 0
                elif s + 1 == len(segs):
                    op, ack = last, 1
                else:
                    op, ack = middle, 0
                plan.append((op, ack, (int(m["psn"]) + s) & 0xFFFFFF,
                             (int(m["remote_va"]) + pos) & 0xFFFFFFFFFFFFFFFF, int(m["reth_len"]), None, sl))
                pos += sl
        assert len(plan) == int(m["npackets"])
        pos = 0
        for s, (op, ack, psn, reth_va, reth_len, imm, sl) in enumerate(plan):
            po = int(m["payload_offset"]) + pos
            payload = np.ascontiguousarray(src[po: po + sl])
            msg = RdmaMsg()
            msg.kind = 0
            msg.opcode = op
            msg.tran_type = int(m["tran_type"])
            msg.solicited = 1 if flags & 0x04 else 0  # RdmaMessageMetaCommon::solicited
            msg.ack_req = ack
            msg.pkey = int(m["msn"])
            msg.dqpn = int(m["dqpn"])
            msg.psn = psn
            msg.reth_va = reth_va
            msg.reth_rkey = int(m["rkey"])
            msg.reth_len = reth_len
            msg.has_imm = 0 if imm is None else 1
            msg.imm = 0 if imm is None else imm
            msg.payload = payload.ctypes.data if sl else None
            msg.payload_len = sl
            rc, pkt = packet_write(msg, int(m["src_ip"]), 4791, int(m["dst_ip"]), 4791, int(m["ip_id"]),
                                   buf_len=max(8192, 128 + sl))
            if rc == LENGTH_TOO_LONG:  # the packetizer reports length 0 and writes nothing
                pos += sl
                continue
            if rc:
                raise ValueError(f"packet_write rc={rc}")
            if flags & 0x01:  # IPv4 checksum filled (responser.rs:198-201 / smoltcp fill_checksum)
                c = ipv4_checksum(pkt[:20])  # bytes 10-11 are 0 as PacketWriter left them
                pkt[10], pkt[11] = c >> 8, c & 0xFF
            icrc = int(pkt[-4:].view("<u4")[0])
            o = int(m["out_offset"]) + s * int(m["slot_stride"])
            wire[o: o + pkt.size] = pkt
            k = int(m["first_packet"]) + s
            lens[k], icrcs[k] = pkt.size, icrc
            pos += sl
    return wire, lens, icrcs


def synth_middle_stream(n: int, *, pmtu: int = 4096, stride: int | None = None,
                        remote_va: int = 0x7F7E8FC00000, reth_len: int = 0, rkey: int = 0x2000003,
                        dqpn: int = 2, psn0: int = 0, msn: int = 0, dst_ip: int = 0xC0A80003,
                        payload_key: int = 0x5EED):
    stride = stride or (28 + 28 + pmtu + 4)
    buf = np.zeros(n * stride, dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint32)
    got = lib().oracle_synth_middle_stream(_ptr(buf), stride, n, _ptr(lens), remote_va, reth_len,
                                           pmtu, rkey, dqpn, psn0, msn, dst_ip, payload_key)
    if got != n:
        raise ValueError(f"synth_middle_stream: rc={got}")
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    return buf, off, lens


def fast_crc32(data, crc: int = 0) -> int:
    a = _as_u8(data)
    return lib().fast_crc32(crc, _ptr(a), a.size)


def fast_compute_icrc(pkt) -> int:
    a = _as_u8(pkt)
    out = ctypes.c_uint32()
    rc = lib().fast_compute_icrc(_ptr(a), a.size, ctypes.byref(out))
    if rc:
        raise ValueError(f"fast_compute_icrc: rc={rc}")
    return out.value


def fast_icrc_strided_timed(base: np.ndarray, stride: int, length: int, n: int, threads: int = 1):
    out = np.zeros(n, dtype=np.uint32)
    secs = lib().fast_icrc_strided_timed(_ptr(base), stride, length, n, _ptr(out), threads)
    return secs, out


def fast_emulator_path_timed(base: np.ndarray, stride: int, length: int, n: int):
    out = np.zeros(n, dtype=np.uint32)
    secs = lib().fast_emulator_path_timed(_ptr(base), stride, length, n, _ptr(out))
    return secs, out


def fast_verify_strided_timed(base: np.ndarray, stride: int, length: int, n: int, threads: int = 1,
                              zero: bool = False):
    """is_icrc_valid over a strided batch (zero=True zeroes the trailers of `base` in place)."""
    ok = np.zeros(n, dtype=np.uint8)
    secs = lib().fast_verify_strided_timed(_ptr(base), stride, length, n, _ptr(ok), threads, 1 if zero else 0)
    return secs, ok


def fast_c0_roundtrip_timed(base: np.ndarray, off, lens, threads: int = 1, reps: int = 1):
    """configs[0]: the emulator's per-packet compute (send) + verify (receive, zeroing) round
    trip over one message's packets, `reps` times on each of `threads` threads.
    Returns (seconds, failed verifies)."""
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    bad = ctypes.c_uint64()
    secs = lib().fast_c0_roundtrip_timed(_ptr(base), _ptr(off), _ptr(lens), off.size, threads, reps,
                                         ctypes.byref(bad))
    return secs, int(bad.value)
