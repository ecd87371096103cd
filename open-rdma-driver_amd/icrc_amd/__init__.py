"""icrc_amd — Python binding of the MI355X ICRC engine (libicrc_amd.so, C-ABI include/icrc.h).

Host-side mirror of the reference's packet/ICRC surface
(blue-rdma-device/src/third_party/net/packet_processor.rs):

    compute_icrc(data) -> int              packet_processor.rs:275-301
    is_icrc_valid(buf) -> bool             packet_processor.rs:341-353 (zeroes the trailer)
    PacketWriter(buf).src_addr(..)...write()   packet_processor.rs:150-265
    write_ip_udp_header(...)               packet_processor.rs:303-332

plus batch / device-resident entry points.  Every CRC runs in the HIP kernel; if the
shared library is missing this module raises at import time (no silent fallback), and
with no GPU every compute call raises IcrcError(ENODEV).
"""
from __future__ import annotations

import atexit
import ctypes
import ipaddress
import os
import weakref
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ICRC_AMD_LIB: another build of the same library (A/B measurements of two builds in one run)
LIB_PATH = os.environ.get("ICRC_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "_build", "libicrc_amd.so")
# The A/B library: the same sources built with ICRC_AB_BUILD (diagnostic variants whose results
# are wrong by design).  Loaded only on request (ab_library()), never by the product
# path.
AB_LIB_PATH = os.environ.get("ICRC_AMD_AB_LIB") or os.path.join(os.path.dirname(_HERE), "_build", "libicrc_amd_ab.so")

OK = 0
EINVAL = -22
ENOMEM = -12
ENODEV = -19
EDEVICE = -5
ETIMEDOUT = -110
ABI_VERSION = 5  # ICRC_ABI_VERSION (include/icrc.h)
HOST_RING, HOST_LAUNCH = 0, 1  # icrc_engine_set_host_path
EBUFFER_NOT_LARGE = -1000
ELENGTH_TOO_LONG = -1001
EINVALID_METADATA = -1002
EINVALID_OPCODE = -1003
MIN_PACKET = 44
ICRC_SIZE = 4
RDMA_PORT = 4791  # blue-rdma-device/src/net.rs:11
LDS_WORDS = 163840 // 4

VERIFY_MISMATCH = 0
VERIFY_OK = 1
VERIFY_BADLEN = 0xFF

_ERRNAMES = {
    EINVAL: "EINVAL", ENOMEM: "ENOMEM", ENODEV: "ENODEV", EDEVICE: "EDEVICE",
    EBUFFER_NOT_LARGE: "BufferNotLargeEnough", ELENGTH_TOO_LONG: "LengthTooLong",
    EINVALID_METADATA: "InvalidMetadataType", EINVALID_OPCODE: "InvalidOpcode",
}


class IcrcError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        self.rc = rc
        super().__init__(f"{what}: {_ERRNAMES.get(rc, rc)} ({rc})")


class RdmaMsg(ctypes.Structure):
    """icrc_rdma_msg — flattened RdmaMessage (third_party/net/types.rs)."""

    _fields_ = [
        ("kind", ctypes.c_uint8), ("opcode", ctypes.c_uint8), ("tran_type", ctypes.c_uint8),
        ("solicited", ctypes.c_uint8), ("ack_req", ctypes.c_uint8), ("aeth_code", ctypes.c_uint8),
        ("aeth_value", ctypes.c_uint8), ("has_imm", ctypes.c_uint8),
        ("has_secondary_reth", ctypes.c_uint8), ("_pad0", ctypes.c_uint8 * 3),
        ("pkey", ctypes.c_uint16), ("_pad1", ctypes.c_uint16), ("dqpn", ctypes.c_uint32),
        ("psn", ctypes.c_uint32), ("msn", ctypes.c_uint32), ("imm", ctypes.c_uint32),
        ("reth_va", ctypes.c_uint64), ("reth_rkey", ctypes.c_uint32), ("reth_len", ctypes.c_uint32),
        ("sec_va", ctypes.c_uint64), ("sec_rkey", ctypes.c_uint32), ("sec_len", ctypes.c_uint32),
        ("payload", ctypes.c_void_p), ("payload_len", ctypes.c_uint64),
    ]


class SynthDesc(ctypes.Structure):
    """icrc_synth_desc (include/icrc.h)."""

    _fields_ = [
        ("offset", ctypes.c_uint64), ("payload_key", ctypes.c_uint64),
        ("payload_pos", ctypes.c_uint64), ("hdr_len", ctypes.c_uint32),
        ("payload_len", ctypes.c_uint32), ("total_len", ctypes.c_uint32),
        ("hdr_index", ctypes.c_uint32),
    ]


SYNTH_DESC_DTYPE = np.dtype([
    ("offset", "<u8"), ("payload_key", "<u8"), ("payload_pos", "<u8"), ("hdr_len", "<u4"),
    ("payload_len", "<u4"), ("total_len", "<u4"), ("hdr_index", "<u4"),
])
assert SYNTH_DESC_DTYPE.itemsize == ctypes.sizeof(SynthDesc) == 40

# icrc_write_msg (include/icrc.h): one RDMA WRITE / READ RESPONSE message for the packetizer.
WRITE_MSG_DTYPE = np.dtype([
    ("local_va", "<u8"), ("remote_va", "<u8"), ("payload_offset", "<u8"), ("out_offset", "<u8"),
    ("total_len", "<u4"), ("reth_len", "<u4"), ("pmtu", "<u4"), ("rkey", "<u4"), ("dqpn", "<u4"),
    ("psn", "<u4"), ("src_ip", "<u4"), ("dst_ip", "<u4"), ("first_packet", "<u4"),
    ("npackets", "<u4"), ("slot_stride", "<u4"), ("msn", "<u2"), ("ip_id", "<u2"),
    ("kind", "u1"), ("tran_type", "u1"), ("flags", "u1"), ("_pad", "u1"), ("lkey", "<u4"),
    ("imm", "<u4"), ("_rsvd", "<u4"),
])
WRITE_FILL_IPV4_CSUM, WRITE_RUST_DRIVER, WRITE_SOLICITED, WRITE_ACK_REQ = 0x01, 0x02, 0x04, 0x08
WRITE_UDP_PAYLOAD_ONLY = 0x10  # BTH .. ICRC at each slot (generate_payload_from_msg's form)
# ToCardWriteDescriptor is_first = false / is_last = false / WriteWithImm (types.rs:548-555, 641-648)
WRITE_NOT_FIRST, WRITE_NOT_LAST, WRITE_WITH_IMM = 0x20, 0x40, 0x80
assert WRITE_MSG_DTYPE.itemsize == 96
MSG_WRITE, MSG_READ_RESPONSE, MSG_READ_REQUEST = 0, 1, 2

# icrc_rx_desc (include/icrc.h): one parsed received packet.
RX_DESC_DTYPE = np.dtype([
    ("reth_va", "<u8"), ("sec_va", "<u8"), ("payload_offset", "<u8"), ("payload_len", "<u4"),
    ("reth_rkey", "<u4"), ("reth_len", "<u4"), ("sec_rkey", "<u4"), ("sec_len", "<u4"),
    ("imm", "<u4"), ("dqpn", "<u4"), ("psn", "<u4"), ("aeth_msn", "<u4"), ("pkey", "<u2"),
    ("opcode", "u1"), ("tran_type", "u1"), ("flags", "u1"), ("pad_cnt", "u1"),
    ("aeth_code", "u1"), ("aeth_value", "u1"), ("icrc_ok", "u1"), ("status", "u1"),
    ("_pad", "u1", (2,)),
])
assert RX_DESC_DTYPE.itemsize == 72
RX_OK, RX_INVALID_OPCODE, RX_INVALID_TRANS_TYPE, RX_TRUNCATED = 0, 1, 2, 3
RX_SOLICITED, RX_ACK_REQ, RX_HAS_IMM, RX_HAS_SECONDARY_RETH, RX_ACKNOWLEDGE = 0x01, 0x02, 0x04, 0x08, 0x10
# icrc_ack_ctx (include/icrc.h): the QP state generate_ack reads (write_first.rs:35-82)
ACK_CTX_DTYPE = np.dtype([("peer_qpn", "<u4"), ("expected_psn", "<u4"), ("flags", "<u4")])
ACK_CTX_QP_VALID = 0x1
ACK_CTX_MR_ERROR = 0x2  # the packet failed its MR / key check (write_first.rs:35): no ACK
ACK_UDP_PAYLOAD_ONLY = 0x1
EMULATOR_SRC_IP = 0xC0A80002  # 192.168.0.2, hard-coded in send_write_message (common.rs:124)


def _load(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"icrc_amd: native library {path} is missing — build it with "
            "`make -C open-rdma-driver_amd` (or __graft_entry__.build()); there is no fallback")
    L = ctypes.CDLL(path)
    vp, u32, u64, i32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
    sig = {
        "icrc_engine_create": (i32, [i32, ctypes.POINTER(vp)]),
        "icrc_engine_destroy": (i32, [vp]),
        "icrc_engine_default": (i32, [i32, ctypes.POINTER(vp)]),
        "icrc_engine_device_ordinal": (i32, [vp]),
        "icrc_engine_stream": (vp, [vp]),
        "icrc_engine_set_kernel_variant": (i32, [vp, i32]),
        "icrc_device_count": (i32, []),
        "icrc_version": (ctypes.c_char_p, []),
        "icrc_compute": (u32, [vp, sz, ctypes.POINTER(i32)]),
        "icrc_verify": (i32, [vp, sz, i32, ctypes.POINTER(i32)]),
        "icrc_compute_batch": (i32, [vp, vp, vp, u32, vp, i32]),
        "icrc_verify_batch": (i32, [vp, vp, vp, u32, vp, i32]),
        "icrc_compute_batch_ex": (i32, [vp, vp, vp, vp, u32, vp, i32]),
        "icrc_verify_batch_ex": (i32, [vp, vp, vp, vp, u32, vp, i32]),
        "icrc_compute_batch_device": (i32, [vp, vp, vp, vp, u32, vp, i32, vp, vp]),
        "icrc_verify_batch_device": (i32, [vp, vp, vp, vp, u32, vp, i32, vp, vp]),
        "icrc_compute_strided_device": (i32, [vp, vp, u64, u32, u32, vp, i32, vp]),
        "icrc_verify_strided_device": (i32, [vp, vp, u64, u32, u32, vp, i32, vp]),
        "icrc_synth_device": (i32, [vp, vp, vp, vp, u32, vp]),
        "icrc_packet_headers": (i32, [vp, sz, ctypes.POINTER(RdmaMsg), u32, ctypes.c_uint16, u32,
                                      ctypes.c_uint16, ctypes.c_uint16, ctypes.POINTER(sz),
                                      ctypes.POINTER(sz)]),
        "icrc_packet_write": (i32, [vp, sz, ctypes.POINTER(RdmaMsg), u32, ctypes.c_uint16, u32,
                                    ctypes.c_uint16, ctypes.c_uint16, ctypes.POINTER(sz)]),
        "icrc_write_ip_udp_header": (None, [vp, u32, ctypes.c_uint16, u32, ctypes.c_uint16,
                                            ctypes.c_uint16, ctypes.c_uint16]),
        "icrc_rdma_header_len": (i32, [ctypes.c_uint8]),
        "icrc_table_image": (i32, [vp, u32]),
        "icrc_table_image_oct": (i32, [vp, u32]),
        "icrc_write_segment_count": (u32, [u64, u32, u32]),
        "icrc_write_packet_len": (u32, [u64, u32, u32, u32]),
        "icrc_write_packetize_device": (i32, [vp, vp, u64, vp, u32, u32, vp, u64, vp, vp, vp]),
        "icrc_rx_parse_device": (i32, [vp, vp, vp, vp, u64, u32, u32, vp, vp, i32, vp, vp]),
        "icrc_ipv4_checksum_device": (i32, [vp, vp, vp, u64, u32, vp, i32, vp]),
        "icrc_ack_from_rx_device": (i32, [vp, vp, vp, u32, vp, u32, vp, u32, vp]),
        "icrc_abi_version": (u32, []),
        "icrc_abi_check": (i32, [u32, sz, sz, sz, sz]),
        "icrc_engine_set_host_path": (i32, [vp, i32]),
        "icrc_engine_host_stats": (i32, [vp, ctypes.POINTER(u64)]),
        "icrc_shutdown": (i32, []),
        "icrc_teardown_stats": (i32, [ctypes.POINTER(u64)]),  # test hook, not in include/icrc.h
        "icrc_ring_selftest": (i32, [i32, i32, i32]),  # test hook, not in include/icrc.h
        "icrc_copy_pool_selftest": (i32, [i32, i32]),  # test hook, not in include/icrc.h
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()
_ab_lib = None
_live_engines: "weakref.WeakSet[Engine]" = weakref.WeakSet()


def _shutdown() -> None:
    """atexit: deterministic teardown before the interpreter, torch and the HIP runtime finalise
    (VERDICT r05 item 1).  Every Engine still open is closed, then icrc_shutdown stops the default
    engines' submission rings, destroys the engines and frees every thread's staging slot, in each
    library loaded; afterwards the library makes no HIP call.  Registered at import: Python runs
    atexit handlers last-in first-out, so this runs before those of modules imported earlier
    (torch)."""
    for eng in list(_live_engines):
        try:
            eng.close()
        except Exception:
            pass
    for L in (lib, _ab_lib):
        if L is not None:
            L.icrc_shutdown()


atexit.register(_shutdown)


def teardown_stats(L: Optional[ctypes.CDLL] = None) -> dict:
    """The library's teardown record (icrc_teardown_stats, a test hook)."""
    out = (ctypes.c_uint64 * 4)()
    _check((L or lib).icrc_teardown_stats(out), "icrc_teardown_stats")
    return {"shutdown": out[0], "engines_destroyed": out[1], "slots_freed": out[2], "refused_after": out[3]}


def ab_library() -> ctypes.CDLL:
    """The A/B build (libicrc_amd_ab.so): for Engine(device, lib=ab_library()) in measurement
    scripts and bench.py's loads-only denominator (variant 19).  Not a product path."""
    global _ab_lib
    if _ab_lib is None:
        _ab_lib = _load(AB_LIB_PATH)
    return _ab_lib


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise IcrcError(rc, what)


_CHAR = ctypes.c_char


def _ptr(a: np.ndarray) -> int:
    """The address of an ndarray's data.  ctypes.c_char.from_buffer is ~4x cheaper than
    a.ctypes.data (which builds a helper object on every access) — the host-message calls take four
    pointers each, and every microsecond spent here is spent holding the GIL, which the other
    Python callers wait for.  Read-only or empty arrays take the ctypes.data path."""
    try:
        return ctypes.addressof(_CHAR.from_buffer(a))
    except (TypeError, ValueError, BufferError):
        return a.ctypes.data


def _u8(a, writable: bool = False) -> np.ndarray:
    """A uint8 view of `a` WITHOUT copying (ndarray, bytearray, memoryview, bytes ...), so that
    in-place effects (is_icrc_valid's trailer zeroing, trailer writes) reach the caller's buffer.
    writable=True raises TypeError for read-only buffers instead of silently writing a copy."""
    if isinstance(a, np.ndarray):
        if a.dtype != np.uint8 or not a.flags.c_contiguous:
            raise TypeError("expected a C-contiguous uint8 array")
        v = a
    else:
        v = np.frombuffer(a, dtype=np.uint8)  # shares memory; read-only for bytes
    if writable and not v.flags.writeable:
        raise TypeError("buffer is read-only, but this call writes into it (trailer)")
    return v


def ip4(addr) -> int:
    """Ipv4Addr -> host-order u32 (a.b.c.d = a<<24|b<<16|c<<8|d)."""
    if isinstance(addr, int):
        return addr
    return int(ipaddress.IPv4Address(addr))


def device_count() -> int:
    return lib.icrc_device_count()


def version() -> str:
    return lib.icrc_version().decode()


COMPACT_WORDS = 1024 + 8192  # kCompactWords: 1024 bulk entries + the 32 KiB final tables


def table_image(width: int = 64, compact: bool = False) -> np.ndarray:
    """The LDS table image the kernels upload for rows of `width` words: 64 (one packet per
    wavefront) or 8 (oct: eight packets per wavefront).  compact: followed by
    the compact form the engine keeps after it in HBM (what the kernels replicate into LDS)."""
    img = np.zeros(LDS_WORDS + (COMPACT_WORDS if compact else 0), dtype=np.uint32)
    fn = {64: lib.icrc_table_image, 8: lib.icrc_table_image_oct}[width]
    _check(fn(img.ctypes.data, img.size), "icrc_table_image")
    return img


# ---- the reference surface -----------------------------------------------------------------
def compute_icrc(data) -> int:
    """compute_icrc (packet_processor.rs:275-301).  Raises IcrcError(EINVAL) where the
    reference would panic (len < 44)."""
    a = _u8(data)
    err = ctypes.c_int(0)
    v = lib.icrc_compute(_ptr(a), a.size, ctypes.byref(err))
    _check(err.value, "compute_icrc")
    return v


def is_icrc_valid(buf, zero_trailer: bool = True) -> bool:
    """is_icrc_valid (packet_processor.rs:341-353): zeroes the trailer in place, as the
    reference does at 350, then recomputes and compares.  `buf` may be any writable buffer
    (ndarray, bytearray, memoryview); a read-only one raises TypeError when zero_trailer."""
    a = _u8(buf, writable=zero_trailer)
    ok = ctypes.c_int(0)
    _check(lib.icrc_verify(_ptr(a), a.size, 1 if zero_trailer else 0, ctypes.byref(ok)),
           "is_icrc_valid")
    return bool(ok.value)


def write_ip_udp_header(buf: np.ndarray, src_addr, src_port: int, dest_addr, dest_port: int,
                        total_length: int, ip_identification: int) -> None:
    """write_ip_udp_header (packet_processor.rs:307-332)."""
    a = _u8(buf, writable=True)
    if a.size < 28:
        raise ValueError("buffer smaller than IPv4+UDP headers")
    lib.icrc_write_ip_udp_header(a.ctypes.data, ip4(src_addr), src_port, ip4(dest_addr), dest_port,
                                 total_length & 0xFFFF, ip_identification & 0xFFFF)


class PacketWriter:
    """PacketWriter builder (packet_processor.rs:150-265).  write() returns the total length
    or raises IcrcError with the PacketProcessorError code."""

    def __init__(self, buf):
        self.buf = _u8(buf, writable=True)
        self._src = self._sport = self._dst = self._dport = self._ipid = self._msg = None

    def src_addr(self, a):
        self._src = ip4(a)
        return self

    def src_port(self, p: int):
        self._sport = p
        return self

    def dest_addr(self, a):
        self._dst = ip4(a)
        return self

    def dest_port(self, p: int):
        self._dport = p
        return self

    def ip_id(self, i: int):
        self._ipid = i
        return self

    def message(self, m: RdmaMsg):
        self._msg = m
        return self

    def write(self) -> int:
        if self._msg is None:
            raise IcrcError(EINVAL, "PacketWriter::write: MissingMessage")
        for name, v in (("MissingIpId", self._ipid), ("MissingSrcAddr", self._src),
                        ("MissingSrcPort", self._sport), ("MissingDestAddr", self._dst),
                        ("MissingDestPort", self._dport)):
            if v is None:
                raise IcrcError(EINVAL, f"PacketWriter::write: {name}")
        n = ctypes.c_size_t(0)
        _check(lib.icrc_packet_write(self.buf.ctypes.data, self.buf.size, ctypes.byref(self._msg),
                                     self._src, self._sport, self._dst, self._dport, self._ipid,
                                     ctypes.byref(n)), "PacketWriter::write")
        return n.value


def packet_headers(msg: RdmaMsg, src, sport: int, dst, dport: int, ip_id: int):
    """Header bytes (IPv4/UDP/BTH/ext) of the packet PacketWriter would build for msg.
    Returns (header uint8 array, total length L)."""
    buf = np.zeros(128, dtype=np.uint8)
    hl = ctypes.c_size_t(0)
    tl = ctypes.c_size_t(0)
    _check(lib.icrc_packet_headers(buf.ctypes.data, buf.size, ctypes.byref(msg), ip4(src), sport,
                                   ip4(dst), dport, ip_id, ctypes.byref(hl), ctypes.byref(tl)),
           "icrc_packet_headers")
    return buf[: hl.value].copy(), tl.value


# ---- batches ---------------------------------------------------------------------------------
def compute_icrc_batch(base: np.ndarray, off, lens, write_trailer: bool = False) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.zeros(off.size, dtype=np.uint32)
    _check(lib.icrc_compute_batch(_ptr(_u8(base, writable=write_trailer)), _ptr(off), _ptr(lens), off.size,
                                  _ptr(out), 1 if write_trailer else 0), "icrc_compute_batch")
    return out


def verify_icrc_batch(base: np.ndarray, off, lens, zero_trailer: bool = False) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    ok = np.zeros(off.size, dtype=np.uint8)
    _check(lib.icrc_verify_batch(_ptr(_u8(base, writable=zero_trailer)), _ptr(off), _ptr(lens), off.size,
                                 _ptr(ok), 1 if zero_trailer else 0), "icrc_verify_batch")
    return ok


def _default_engine(device: int = -1) -> ctypes.c_void_p:
    h = ctypes.c_void_p()
    _check(lib.icrc_engine_default(device, ctypes.byref(h)), "icrc_engine_default")
    return h


def set_host_path(path: int, device: int = -1) -> None:
    """The default engine's host-message path (the module-level drop-ins above use it):
    HOST_RING (default) or HOST_LAUNCH."""
    _check(lib.icrc_engine_set_host_path(_default_engine(device), path), "icrc_engine_set_host_path")


def host_stats(device: int = -1) -> dict:
    """The default engine's submission-ring counters (icrc_engine_host_stats)."""
    out = (ctypes.c_uint64 * 4)()
    _check(lib.icrc_engine_host_stats(_default_engine(device), out), "icrc_engine_host_stats")
    return {"jobs": out[0], "launches": out[1], "relaunches": out[2], "timeouts": out[3]}


def abi_check() -> int:
    """icrc_abi_check with this binding's own struct sizes (the mirrors below)."""
    return lib.icrc_abi_check(ABI_VERSION, WRITE_MSG_DTYPE.itemsize, RX_DESC_DTYPE.itemsize, 12, SYNTH_DESC_DTYPE.itemsize)


def ring_selftest(scenario: int, threads: int = 3, jobs_per_thread: int = 200) -> int:
    """The submission ring's host protocol against a simulated service kernel on a CPU thread
    (icrc_ring_selftest, a test hook of the library): 0 = the scenario behaved as specified."""
    return lib.icrc_ring_selftest(scenario, threads, jobs_per_thread)


def copy_pool_selftest(threads: int = 4, jobs: int = 200) -> int:
    """The host copy pool that gathers pageable host batches (icrc_copy_pool_selftest, a test
    hook): callers running jobs at once, every task exactly once per job.  0 = as specified."""
    return lib.icrc_copy_pool_selftest(threads, jobs)


class Engine:
    """One engine per GPU (icrc_engine_create).  Device entry points take raw device pointers
    (e.g. torch tensor .data_ptr()) and a hipStream_t handle (e.g.
    torch.cuda.current_stream().cuda_stream); 0/None = the HIP null stream (torch's default
    stream), engine.stream = the engine's own non-blocking stream."""

    def __init__(self, device: int = 0, lib: Optional[ctypes.CDLL] = None):
        self._lib = lib or globals()["lib"]
        h = ctypes.c_void_p()
        _check(self._lib.icrc_engine_create(device, ctypes.byref(h)), "icrc_engine_create")
        self.handle = h
        self.device = device
        self.stream = self._lib.icrc_engine_stream(h) or 0
        _live_engines.add(self)

    @property
    def ordinal(self) -> int:
        """The HIP device the engine runs on (icrc_engine_device_ordinal)."""
        return int(self._lib.icrc_engine_device_ordinal(self.handle))

    def set_host_path(self, path: int) -> None:
        """HOST_RING (default: the submission ring) or HOST_LAUNCH (a kernel launch per message)."""
        _check(self._lib.icrc_engine_set_host_path(self.handle, path), "icrc_engine_set_host_path")

    def host_stats(self) -> dict:
        """The submission ring's counters (icrc_engine_host_stats)."""
        out = (ctypes.c_uint64 * 4)()
        _check(self._lib.icrc_engine_host_stats(self.handle, out), "icrc_engine_host_stats")
        return {"jobs": out[0], "launches": out[1], "relaunches": out[2], "timeouts": out[3]}

    def set_variant(self, variant: int) -> None:
        """Kernel variant for A/B runs (0 = unpipelined, S >= 1 = S packets in flight/wave)."""
        _check(self._lib.icrc_engine_set_kernel_variant(self.handle, variant), "set_kernel_variant")

    def close(self) -> None:
        """icrc_engine_destroy (idempotent; after icrc_shutdown the library has already destroyed it
        and refuses the handle with EINVAL)."""
        if self.handle:
            h, self.handle = self.handle, None
            self._lib.icrc_engine_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compute_strided(self, d_base: int, stride: int, length: int, n: int, d_out: int,
                        write_trailer: bool = False, stream: Optional[int] = None) -> None:
        _check(self._lib.icrc_compute_strided_device(self.handle, d_base, stride, length, n, d_out,
                                               1 if write_trailer else 0, stream or None),
               "icrc_compute_strided_device")

    def verify_strided(self, d_base: int, stride: int, length: int, n: int, d_ok: int,
                       zero_trailer: bool = False, stream: Optional[int] = None) -> None:
        _check(self._lib.icrc_verify_strided_device(self.handle, d_base, stride, length, n, d_ok,
                                              1 if zero_trailer else 0, stream or None),
               "icrc_verify_strided_device")

    def compute_batch(self, d_base: int, d_off: int, d_len: int, n: int, d_out: int,
                      write_trailer: bool = False, d_nerr: int = 0,
                      stream: Optional[int] = None) -> None:
        _check(self._lib.icrc_compute_batch_device(self.handle, d_base, d_off, d_len, n, d_out or None,
                                             1 if write_trailer else 0, d_nerr or None,
                                             stream or None), "icrc_compute_batch_device")

    def verify_batch(self, d_base: int, d_off: int, d_len: int, n: int, d_ok: int,
                     zero_trailer: bool = False, d_nerr: int = 0,
                     stream: Optional[int] = None) -> None:
        _check(self._lib.icrc_verify_batch_device(self.handle, d_base, d_off, d_len, n, d_ok,
                                            1 if zero_trailer else 0, d_nerr or None,
                                            stream or None), "icrc_verify_batch_device")

    def synth(self, d_base: int, d_desc: int, d_hdr: int, n: int,
              stream: Optional[int] = None) -> None:
        _check(self._lib.icrc_synth_device(self.handle, d_base, d_desc, d_hdr, n, stream or None),
               "icrc_synth_device")

    def compute_batch_host(self, base: np.ndarray, off, lens, write_trailer: bool = False):
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros(off.size, dtype=np.uint32)
        _check(self._lib.icrc_compute_batch_ex(self.handle, _u8(base, writable=write_trailer).ctypes.data, off.ctypes.data,
                                         lens.ctypes.data, off.size, out.ctypes.data,
                                         1 if write_trailer else 0), "icrc_compute_batch_ex")
        return out

    def verify_batch_host(self, base: np.ndarray, off, lens, zero_trailer: bool = False) -> np.ndarray:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        ok = np.zeros(off.size, dtype=np.uint8)
        _check(self._lib.icrc_verify_batch_ex(self.handle, _u8(base, writable=zero_trailer).ctypes.data, off.ctypes.data,
                                        lens.ctypes.data, off.size, ok.ctypes.data,
                                        1 if zero_trailer else 0), "icrc_verify_batch_ex")
        return ok

    def rx_parse(self, d_base: int, d_off: int, d_len: int, n: int, d_desc: int, d_ok: int = 0,
                 zero_trailer: bool = False, d_nerr: int = 0, stride: int = 0, length: int = 0,
                 stream: Optional[int] = None) -> None:
        """Fused receive (icrc_rx_parse_device): verify + strip + parse into RX_DESC_DTYPE."""
        _check(self._lib.icrc_rx_parse_device(self.handle, d_base, d_off or None, d_len or None, stride, length, n,
                                        d_desc, d_ok or None, 1 if zero_trailer else 0, d_nerr or None,
                                        stream or None), "icrc_rx_parse_device")

    def ipv4_checksum(self, d_base: int, n: int, d_off: int = 0, stride: int = 0, d_csum: int = 0,
                      fill: bool = False, stream: Optional[int] = None) -> None:
        """Batched IPv4 header checksum (icrc_ipv4_checksum_device, responser.rs:321-338)."""
        _check(self._lib.icrc_ipv4_checksum_device(self.handle, d_base, d_off or None, stride, n, d_csum or None,
                                             1 if fill else 0, stream or None), "icrc_ipv4_checksum_device")

    def ack_from_rx(self, d_desc: int, d_ctx: int, n: int, d_out: int, out_stride: int = 48, d_out_len: int = 0,
                    udp_payload_only: bool = False, stream: Optional[int] = None) -> None:
        """Receive-side auto-ACK (icrc_ack_from_rx_device, generate_ack net/util.rs:134-170)."""
        _check(self._lib.icrc_ack_from_rx_device(self.handle, d_desc, d_ctx, n, d_out, out_stride, d_out_len or None,
                                           ACK_UDP_PAYLOAD_ONLY if udp_payload_only else 0, stream or None),
               "icrc_ack_from_rx_device")

    def packetize(self, d_src: int, src_bytes: int, d_msgs: int, nmsgs: int, npackets: int,
                  d_wire: int, wire_bytes: int, d_pkt_len: int = 0, d_icrc: int = 0,
                  stream: Optional[int] = None) -> None:
        """Fused send step (icrc_write_packetize_device): segment, serialise, copy, pad, ICRC."""
        _check(self._lib.icrc_write_packetize_device(self.handle, d_src or None, src_bytes, d_msgs, nmsgs,
                                               npackets, d_wire, wire_bytes, d_pkt_len or None,
                                               d_icrc or None, stream or None),
               "icrc_write_packetize_device")


def write_segment_count(local_va: int, total_len: int, pmtu: int) -> int:
    """generate_segments_from_request(...).len() (common.rs:152-176)."""
    return int(lib.icrc_write_segment_count(local_va, total_len, pmtu))


def write_packet_len(local_va: int, total_len: int, pmtu: int, s: int) -> int:
    """Wire length of segment s of a WRITE / READ RESPONSE message (0 past the last)."""
    return int(lib.icrc_write_packet_len(local_va, total_len, pmtu, s))


def write_messages(specs, slot_stride: int = 0, base_out: int = 0) -> np.ndarray:
    """Build an icrc_write_msg array from dicts (local_va, remote_va, payload_offset,
    total_len, pmtu, ...), filling first_packet / npackets / out_offset so the messages' packets
    are laid out back to back (slot_stride 0 = each message's pmtu + 64, 4-byte aligned)."""
    msgs = np.zeros(len(specs), dtype=WRITE_MSG_DTYPE)
    first, out = 0, base_out
    for i, s in enumerate(specs):
        m = msgs[i]
        for k, v in s.items():
            m[k] = v
        if "src_ip" not in s:
            m["src_ip"] = EMULATOR_SRC_IP
        if "reth_len" not in s:
            m["reth_len"] = s["total_len"]
        if "ip_id" not in s:
            m["ip_id"] = 1  # generate_payload_from_msg (net/util.rs:179)
        if int(s.get("kind", 0)) == MSG_READ_REQUEST:
            n = 1  # Read::handle sends one request packet (read.rs:33-89)
        else:
            seg_va = s.get("remote_va", 0) if int(s.get("flags", 0)) & WRITE_RUST_DRIVER else s.get("local_va", 0)
            n = write_segment_count(int(seg_va), int(s["total_len"]), int(s["pmtu"]))
        stride = int(s.get("slot_stride", slot_stride or max(128, (int(s.get("pmtu", 0)) + 64 + 3) & ~3)))
        m["npackets"], m["first_packet"], m["slot_stride"] = n, first, stride
        if "out_offset" not in s:
            m["out_offset"] = out
        out = int(m["out_offset"]) + n * stride
        first += n
    return msgs


from . import workloads  # noqa: E402,F401  (synthetic packet streams)
