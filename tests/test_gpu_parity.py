"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle, bit-exact.

Oracle = oracle/icrc_oracle.c (restatement of packet_processor.rs:275-353), pinned by the
reference KATs in tests/golden_kats.py and the zlib fixtures in tests/golden/.
"""
import numpy as np
import pytest

import oracle
from golden_kats import KATS, KAT1, KAT1_ICRC

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def stream_handle():
    return torch.cuda.current_stream().cuda_stream


def oracle_icrcs(buf: np.ndarray, off, lens):
    return oracle.compute_icrc_batch(buf, np.asarray(off, np.uint64), np.asarray(lens, np.uint32))


def run_batch(engine, buf: np.ndarray, off, lens, write_trailer=False):
    d_buf = dev(buf)
    d_off = dev(np.asarray(off, np.uint64))
    d_len = dev(np.asarray(lens, np.uint32))
    n = len(lens)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_nerr = torch.zeros(1, dtype=torch.int32, device="cuda")
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(),
                         write_trailer=write_trailer, d_nerr=d_nerr.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    return (d_out.cpu().numpy().view(np.uint32), int(d_nerr.item()), d_buf.cpu().numpy())


def test_kats_scalar_dropin():
    import icrc_amd

    for pkt, want in KATS:
        assert icrc_amd.compute_icrc(pkt) == want


def test_kats_device_batch(engine):
    bufs = [np.frombuffer(p, np.uint8) for p, _ in KATS]
    off = np.cumsum([0] + [b.size for b in bufs[:-1]]).astype(np.uint64)
    buf = np.concatenate(bufs)
    out, nerr, _ = run_batch(engine, buf, off, [b.size for b in bufs])
    assert nerr == 0
    assert [int(x) for x in out] == [w for _, w in KATS]


def test_strided_write_middle_stream(engine):
    n = 2048
    buf, off, lens = oracle.synth_middle_stream(n)
    L = int(lens[0])
    d_buf = dev(buf)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, oracle_icrcs(buf, off, lens))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ragged_any_length_any_alignment(engine, seed):
    """Lengths 44..9000 (all residues mod 4) at random byte offsets: exercises the generic
    path (misaligned / L % 4 != 0) and the fast path in one launch."""
    rng = np.random.default_rng(seed)
    n = 3000
    lens = rng.integers(44, 9000, n).astype(np.uint32)
    lens[:64] = np.arange(44, 108)             # every short length
    gaps = rng.integers(0, 8, n)
    if seed == 0:
        gaps[:] = 0                               # packed, mostly misaligned
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1].astype(np.uint64))
    total = int(off[-1] + lens[-1])
    buf = rng.integers(0, 256, total + 16, dtype=np.uint8)
    out, nerr, _ = run_batch(engine, buf, off, lens)
    assert nerr == 0
    np.testing.assert_array_equal(out, oracle_icrcs(buf, off, lens))


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 10, 11, 12])
def test_every_kernel_variant_is_bit_exact(engine, variant):
    """The A/B variants (unpipelined, S chains x D-deep prefetch) on a ragged batch with
    misaligned and over-long packets and on a strided stream."""
    rng = np.random.default_rng(100 + variant)
    n = 1500
    lens = rng.choice([44, 48, 316, 1084, 4156, 4157, 5000, 9000], n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 2, n - 1).astype(np.uint64) * 4
                        + (rng.random(n - 1) < 0.05))
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    engine.set_variant(variant)
    try:
        out, nerr, _ = run_batch(engine, buf, off, lens)
        assert nerr == 0
        np.testing.assert_array_equal(out, oracle_icrcs(buf, off, lens))
        sbuf, soff, slens = oracle.synth_middle_stream(777)
        L = int(slens[0])
        d = dev(sbuf)
        d_out = torch.zeros(777, dtype=torch.int32, device="cuda")
        engine.compute_strided(d.data_ptr(), L, L, 777, d_out.data_ptr(), stream=stream_handle())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), oracle_icrcs(sbuf, soff, slens))
    finally:
        engine.set_variant(-1)


def test_max_and_boundary_lengths(engine):
    rng = np.random.default_rng(7)
    lens = np.array([44, 47, 48, 255, 256, 257, 259, 260, 1023, 1024, 1028, 4156, 4160, 8192,
                     16384, 65532, 65535], dtype=np.uint32)
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(((lens[:-1].astype(np.uint64) + 3) // 4) * 4)
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 4, dtype=np.uint8)
    out, nerr, _ = run_batch(engine, buf, off, lens)
    assert nerr == 0
    np.testing.assert_array_equal(out, oracle_icrcs(buf, off, lens))


def test_short_lengths_are_errors_not_panics(engine):
    rng = np.random.default_rng(3)
    lens = np.array([0, 4, 43, 44, 100], dtype=np.uint32)
    off = np.arange(lens.size, dtype=np.uint64) * 128
    buf = rng.integers(0, 256, 128 * lens.size, dtype=np.uint8)
    out, nerr, _ = run_batch(engine, buf, off, lens)
    assert nerr == 3
    assert list(out[:3]) == [0, 0, 0]
    np.testing.assert_array_equal(out[3:], oracle_icrcs(buf, off[3:], lens[3:]))


def test_write_trailer_then_verify_with_negatives(engine):
    """C3-style round trip: compute (send) writes trailers, verify (recv) over the same
    buffer; then one flipped bit per 64 packets must fail exactly there."""
    import icrc_amd

    w = icrc_amd.workloads.write_message(1 << 20, 4096)
    d_hdr = dev(w.hdr)
    d_desc = dev(w.desc.view(np.uint8))
    d_buf = torch.zeros(w.total_bytes + 64, dtype=torch.uint8, device="cuda")
    s = stream_handle()
    engine.synth(d_buf.data_ptr(), d_desc.data_ptr(), d_hdr.data_ptr(), w.n, stream=s)
    d_off, d_len = dev(w.off), dev(w.lens)
    d_out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_out.data_ptr(),
                         write_trailer=True, stream=s)
    d_ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_ok.data_ptr(),
                        stream=s)
    torch.cuda.synchronize()
    assert bool((d_ok == 1).all())
    host = d_buf.cpu().numpy()
    # trailers equal the oracle's ICRCs and the whole packets equal the oracle's PacketWriter
    ref_buf, ref_off, ref_lens = oracle.synth_write(
        1 << 20, 4096, local_va=0x7F7E8EE00000, remote_va=0x7F7E8FC00000, rkey=0x2000003, dqpn=2,
        psn0=0, msn=0, dst_ip=0xC0A80003, payload_key=0xABCDEF)
    assert ref_lens.tolist() == w.lens.tolist()
    for i in range(w.n):
        a = host[int(w.off[i]): int(w.off[i]) + int(w.lens[i])]
        b = ref_buf[int(ref_off[i]): int(ref_off[i]) + int(ref_lens[i])]
        np.testing.assert_array_equal(a, b)
    # negative control
    flip = np.arange(0, w.n, 64)
    rng = np.random.default_rng(11)
    for i in flip:
        pos = int(w.off[i]) + int(rng.integers(0, int(w.lens[i])))
        host[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    d_buf2 = dev(host)
    d_ok.zero_()
    engine.verify_batch(d_buf2.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_ok.data_ptr(),
                        zero_trailer=True, stream=s)
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy()
    expect = np.ones(w.n, np.uint8)
    for i in flip:
        # a flip inside a masked header byte (1, 8, 10, 11, 26, 27, 32) or the trailer
        # compares against the oracle instead of assuming a mismatch
        pkt = host[int(w.off[i]): int(w.off[i]) + int(w.lens[i])].copy()
        expect[i] = 1 if oracle.is_icrc_valid(pkt) else 0
    np.testing.assert_array_equal(ok, expect)
    trailers = d_buf2.cpu().numpy()
    for i in range(w.n):
        end = int(w.off[i]) + int(w.lens[i])
        assert not trailers[end - 4: end].any()  # zero_trailer, packet_processor.rs:350


def test_synth_c1_matches_oracle_bytes(engine):
    import icrc_amd

    n = 256
    w = icrc_amd.workloads.write_middle_stream(n, reth_len=0)
    d_buf = icrc_amd.workloads.synthesize(engine, w, stream=stream_handle())
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_strided(d_buf.data_ptr(), w.stride, int(w.lens[0]), n, d_out.data_ptr(),
                           write_trailer=True, stream=stream_handle())
    torch.cuda.synchronize()
    ref, ref_off, ref_lens = oracle.synth_middle_stream(n, payload_key=0x5EED5EED, reth_len=0)
    np.testing.assert_array_equal(d_buf.cpu().numpy(), ref)


def test_mixed_mtu_stream(engine):
    import icrc_amd

    w = icrc_amd.workloads.mixed_mtu_stream(20000)
    d_buf = icrc_amd.workloads.synthesize(engine, w, stream=stream_handle())
    out, nerr, host = run_batch(engine, d_buf.cpu().numpy(), w.off, w.lens)
    assert nerr == 0
    np.testing.assert_array_equal(out, oracle_icrcs(host, w.off, w.lens))
    pads = (4 - w.desc["payload_len"] % 4) % 4
    assert set(np.unique(pads).tolist()) == {0, 1, 2, 3}


def test_host_batch_and_scalar_surface():
    import icrc_amd

    rng = np.random.default_rng(5)
    buf, off, lens = oracle.synth_middle_stream(64, pmtu=1024)
    got = icrc_amd.compute_icrc_batch(buf, off, lens, write_trailer=True)
    np.testing.assert_array_equal(got, oracle_icrcs(buf, off, lens))
    ok = icrc_amd.verify_icrc_batch(buf, off, lens)
    assert ok.all()
    pkt = np.frombuffer(KAT1, np.uint8).copy()
    assert icrc_amd.is_icrc_valid(pkt)
    assert not pkt[-4:].any()                  # zeroed in place like the reference
    pkt[100] ^= 1
    assert not icrc_amd.is_icrc_valid(pkt)
    with pytest.raises(icrc_amd.IcrcError):
        icrc_amd.compute_icrc(np.zeros(43, np.uint8))
    for L in (44, 45, 46, 47, 1000, 1001):
        p = rng.integers(0, 256, L, dtype=np.uint8)
        assert icrc_amd.compute_icrc(p) == oracle.compute_icrc(p)


@pytest.mark.parametrize("pinned", [False, True])
def test_host_batch_multi_chunk(engine, pinned):
    """Host-resident path over several 64 MiB chunks (two pipelined stages), pinned (direct
    span copies) and pageable (gathered), with write_trailer applied to the host buffer."""
    n = 20000
    buf, off, lens = oracle.synth_middle_stream(n)
    want = oracle_icrcs(buf, off, lens)
    if pinned:
        t = torch.empty(buf.size, dtype=torch.uint8, pin_memory=True)
        host = t.numpy()
        host[:] = buf
    else:
        host = buf.copy()
    host[np.asarray(off + lens.astype(np.uint64) - 4, np.int64)[:, None] + np.arange(4)] = 0
    got = engine.compute_batch_host(host, off, lens, write_trailer=True)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(host, buf)  # trailers written back == the oracle's packets


def test_packet_writer_matches_oracle():
    import icrc_amd

    rng = np.random.default_rng(9)
    for opcode in (0x06, 0x07, 0x08, 0x0A, 0x0D, 0x0E, 0x0F, 0x10, 0x09, 0x0B, 0x0C, 0x11):
        for plen in (0, 1, 2, 3, 4, 129):
            payload = rng.integers(0, 256, max(plen, 1), dtype=np.uint8)
            m1, m2 = icrc_amd.RdmaMsg(), oracle.RdmaMsg()
            for m in (m1, m2):
                m.kind = 1 if opcode == 0x11 else 0
                m.opcode = opcode
                m.solicited = 1
                m.ack_req = 1
                m.pkey = 0x1234
                m.dqpn = 0xABCDEF
                m.psn = 0x123456
                m.msn = 77
                m.aeth_value = 0x1F
                m.reth_va = 0x1122334455667788
                m.reth_rkey = 0xDEADBEEF
                m.reth_len = 0x10000
                m.has_imm = 1
                m.imm = 0xCAFEBABE
                m.has_secondary_reth = 1
                m.sec_va = 0x99
                m.sec_rkey = 0x77
                m.sec_len = 0x55
                m.payload = payload.ctypes.data
                m.payload_len = plen
            buf = np.zeros(8192, np.uint8)
            L = icrc_amd.PacketWriter(buf).src_addr("192.168.0.2").src_port(4791).dest_addr(
                "192.168.0.3").dest_port(4791).ip_id(1).message(m1).write()
            rc, ref = oracle.packet_write(m2, 0xC0A80002, 4791, 0xC0A80003, 4791, 1)
            assert rc == 0
            np.testing.assert_array_equal(buf[:L], ref)


@pytest.mark.parametrize("n", [1 << 20])
def test_full_size_c1_properties(engine, n):
    """BASELINE configs[1] at full size (1 Mi x 4156 B): device ICRCs equal the CPU port's on
    the same bytes (the pclmul port is itself checked against the oracle in the CPU suite),
    and compute -> write trailer -> verify round-trips for every packet."""
    import icrc_amd

    w = icrc_amd.workloads.write_middle_stream(n)
    L = int(w.lens[0])
    s = stream_handle()
    d_buf = icrc_amd.workloads.synthesize(engine, w, stream=s)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), write_trailer=True, stream=s)
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_strided(d_buf.data_ptr(), L, L, n, d_ok.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert bool((d_ok == 1).all())
    host = d_buf.cpu().numpy()
    _, cpu = oracle.fast_icrc_strided_timed(host, L, L, n, threads=16)
    np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), cpu)
    # spot-check a sample against the plain oracle itself
    idx = np.random.default_rng(1).integers(0, n, 512)
    np.testing.assert_array_equal(
        d_out.cpu().numpy().view(np.uint32)[idx],
        oracle_icrcs(host, idx.astype(np.uint64) * np.uint64(L), np.full(idx.size, L, np.uint32)))
