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


@pytest.mark.parametrize("variant", [0, 13, 16, 17, 40])
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
        want = oracle_icrcs(sbuf, soff, slens)
        np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), want)
        # the trailer-storing instantiations: write_trailer, then verify with zero_trailer
        d.view(777, L)[:, L - 4:] = 0x5A
        engine.compute_strided(d.data_ptr(), L, L, 777, d_out.data_ptr(), write_trailer=True, stream=stream_handle())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d.view(777, L)[:, L - 4:].contiguous().cpu().numpy().view("<u4").ravel(), want)
        d_ok = torch.zeros(777, dtype=torch.uint8, device="cuda")
        d.view(777, L)[5, 100] ^= 1  # one corrupted packet
        engine.verify_strided(d.data_ptr(), L, L, 777, d_ok.data_ptr(), zero_trailer=True, stream=stream_handle())
        torch.cuda.synchronize()
        ok = d_ok.cpu().numpy()
        assert ok[5] == 0 and ok.sum() == 776
        assert not d.view(777, L)[:, L - 4:].any().item()
        # ragged verify (and zeroing) through this variant
        hb = buf.copy()
        tr = (off + lens.astype(np.uint64) - 4).astype(np.int64)[:, None] + np.arange(4)
        hb[tr] = oracle_icrcs(buf, off, lens).view(np.uint8).reshape(-1, 4)
        d_b, d_o, d_l = dev(hb), dev(off), dev(lens)
        d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        engine.verify_batch(d_b.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), n, d_ok.data_ptr(), zero_trailer=True,
                            stream=stream_handle())
        torch.cuda.synchronize()
        assert bool((d_ok == 1).all())
        assert not d_b.cpu().numpy()[tr].any()
    finally:
        engine.set_variant(-1)


def _block_mix(rng, nblocks=48):
    """Blocks of 64 packets of contrasting shapes for the oct kernel's block / set / frame
    logic: tiny 1-row packets (16 sets of 1 row per block: the load side outruns the process
    side and stalls), blocks with no fast-path packet at all (misaligned), partial sets, one
    jumbo packet among short ones, unsorted mixed MTUs."""
    lens, gaps = [], []
    for b in range(nblocks):
        kind = b % 6
        if kind == 0:
            ln, gp = rng.choice([44, 48, 52, 60, 64], 64), np.zeros(64, int)
        elif kind == 1:
            ln, gp = rng.choice([316, 1084], 64), np.ones(64, int)       # misaligned: generic path
        elif kind == 2:
            ln, gp = rng.choice([316, 1084, 4156], 64), np.zeros(64, int)
            gp[rng.integers(0, 64, 5)] = 1                               # a few irregular
        elif kind == 3:
            ln, gp = np.full(64, 316), np.zeros(64, int)
            ln[17] = 9000                                                # jumbo among short
        elif kind == 4:
            ln, gp = rng.integers(11, 1100, 64) * 4, np.zeros(64, int)  # every row count
        else:
            ln, gp = np.full(64, 4156), np.zeros(64, int)
        lens.append(ln)
        gaps.append(gp)
    lens = np.concatenate(lens).astype(np.uint32)
    gaps = np.concatenate(gaps).astype(np.uint64)
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    return off, lens


@pytest.mark.parametrize("variant", [-1, 40, 140, 240])
@pytest.mark.parametrize("n", [3072, 1000, 37])
def test_block_transitions_compute_verify(engine, variant, n):
    """The oct kernel (40) and the hybrid dispatch (-1: oct for L <= 1088, the one-packet pipeline
    for the rest, or at these sizes the one-packet pipeline alone; 140: the split forced as two
    kernels; 240: with the compacting long-packet walker) on contrasting 64-packet blocks: compute with trailer
    write, then verify (all ok), then negatives (one flipped bit per 7 packets) with in-place
    trailer zeroing."""
    rng = np.random.default_rng((variant % 100 + 2) * 1000 + n)
    off, lens = _block_mix(rng)
    off, lens = off[:n], lens[:n]
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    engine.set_variant(variant)
    try:
        out, nerr, wrote = run_batch(engine, buf, off, lens, write_trailer=True)
        assert nerr == 0
        want = oracle_icrcs(buf, off, lens)
        np.testing.assert_array_equal(out, want)
        for i in range(0, n, 97):
            t = int(off[i] + lens[i] - 4)
            assert int(wrote[t: t + 4].view(np.uint32)[0]) == int(want[i])
        bad = np.arange(0, n, 7)
        for i in bad:
            wrote[int(off[i]) + 36 + int(rng.integers(0, int(lens[i]) - 40))] ^= 0x10  # ICRC-covered, unmasked
        d_buf = dev(wrote)
        d_off, d_len = dev(off), dev(lens)
        d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(),
                            zero_trailer=True, stream=stream_handle())
        torch.cuda.synchronize()
        ok = d_ok.cpu().numpy()
        expect = np.ones(n, np.uint8)
        expect[bad] = 0
        np.testing.assert_array_equal(ok, expect)
        after = d_buf.cpu().numpy()
        for i in range(0, n, 53):
            t = int(off[i] + lens[i] - 4)
            assert not after[t: t + 4].any()
    finally:
        engine.set_variant(-1)


def test_split_batch_dense_and_sparse_waves(engine):
    """Hybrid dispatch at a size where every wave owns whole 64-packet blocks: waves whose first
    block is mostly long take the dense long-packet pipeline (short packets as empty slots), the
    others the compacting walker; workgroups with no short packet skip the oct kernel.  Blocks of
    64: all long / long with a few short and irregular packets / mostly short / all short, in runs
    so that whole workgroups are all long.  Compute with trailer write, then verify with negatives."""
    rng = np.random.default_rng(4242)
    nblk = 5000  # 320 000 packets: > 64 per wave on a 256-CU grid
    kinds = np.repeat(rng.integers(0, 4, nblk // 40), 40)[:nblk]
    kinds[:1200] = 0  # the first workgroups: long packets only
    lens, gaps = [], []
    for k in kinds:
        if k == 0:
            ln, gp = rng.choice([2048, 2052, 3000, 4156], 64), np.zeros(64, int)
        elif k == 1:
            ln, gp = np.full(64, 4156), np.zeros(64, int)
            ln[rng.integers(0, 64, 6)] = rng.choice([44, 316, 1084], 6)
            gp[rng.integers(0, 64, 2)] = 1  # irregular offsets
            ln[rng.integers(0, 64, 1)] = 4157  # L % 4 != 0
        elif k == 2:
            ln, gp = rng.choice([60, 316, 1084], 64), np.zeros(64, int)
            ln[rng.integers(0, 64, 2)] = 4156
        else:
            ln, gp = rng.integers(11, 511, 64) * 4, np.zeros(64, int)
        lens.append(ln)
        gaps.append(gp)
    lens = np.concatenate(lens).astype(np.uint32)
    gaps = np.concatenate(gaps).astype(np.uint64)
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    n = lens.size
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    out, nerr, wrote = run_batch(engine, buf, off, lens, write_trailer=True)
    assert nerr == 0
    want = oracle_icrcs(buf, off, lens)
    np.testing.assert_array_equal(out, want)
    bad = np.arange(0, n, 101)
    for i in bad:
        wrote[int(off[i]) + 36 + int(rng.integers(0, int(lens[i]) - 40))] ^= 0x04
    d_buf, d_off, d_len = dev(wrote), dev(off), dev(lens)
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(),
                        zero_trailer=True, stream=stream_handle())
    torch.cuda.synchronize()
    expect = np.ones(n, np.uint8)
    expect[bad] = 0
    np.testing.assert_array_equal(d_ok.cpu().numpy(), expect)
    # zero_trailer (deferred trailer pass at this size): every trailer zeroed, nothing else touched
    after = d_buf.cpu().numpy()
    tpos = (off + lens.astype(np.uint64) - 4).astype(np.int64)
    idx = tpos[:, None] + np.arange(4)[None, :]
    assert not after[idx].any()
    keep = np.ones(after.size, bool)
    keep[idx.ravel()] = False
    np.testing.assert_array_equal(after[keep], wrote[keep])


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


@pytest.mark.parametrize("pinned", [False, True])
def test_host_message_batches_three_threads(pinned):
    """One-message host batches (at most 1024 packets / 8 MiB: the submitter path, zero-copy from
    pinned buffers, combined across threads) from three threads at once, as the emulator's send,
    packet-handler and receive threads would call them: configs[0]-shaped WRITE messages and ragged
    misaligned batches, compute with write_trailer then verify with zero_trailer, one corrupted
    packet per batch; plus 1024 / 1025-packet batches on both sides of the size switch."""
    import threading

    import icrc_amd

    def buffer(a):
        if not pinned:
            return a.copy()
        t = torch.empty(a.size, dtype=torch.uint8, pin_memory=True)
        h = t.numpy()
        h[:] = a
        keep.append(t)
        return h

    keep, errors = [], []

    def run(seed):
        try:
            rng = np.random.default_rng(seed)
            for it in range(12):
                if it % 3 == 0:
                    ref, off, lens = oracle.synth_write(256 << 10, 4096, local_va=0x7F7E8EE00000 + it * 4,
                                                        remote_va=0x7F7E8FC00000, rkey=3, dqpn=2 + seed, psn0=it,
                                                        msn=0, dst_ip=0xC0A80003, payload_key=seed * 100 + it)
                else:
                    n = int(rng.integers(1, 300))
                    lens = rng.integers(44, 9000, n).astype(np.uint32)
                    off = np.zeros(n, np.uint64)
                    off[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 5, n - 1).astype(np.uint64))
                    ref = rng.integers(0, 256, int(off[-1] + lens[-1]) + 3, dtype=np.uint8)
                want = oracle_icrcs(ref, off, lens)
                host = buffer(ref)
                got = icrc_amd.compute_icrc_batch(host, off, lens, write_trailer=True)
                np.testing.assert_array_equal(got, want)
                bad = int(rng.integers(0, len(lens)))
                host[int(off[bad]) + 40 + int(rng.integers(0, int(lens[bad]) - 44))] ^= 0x40
                ok = icrc_amd.verify_icrc_batch(host, off, lens, zero_trailer=True)
                expect = np.ones(len(lens), np.uint8)
                expect[bad] = 0
                np.testing.assert_array_equal(ok, expect)
                tr = (off + lens.astype(np.uint64) - 4).astype(np.int64)[:, None] + np.arange(4)
                assert not host[tr].any()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ths = [threading.Thread(target=run, args=(k,)) for k in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors, errors
    for n in (1024, 1025):  # the largest submitter batch, and the staged path
        ref, off, lens = oracle.synth_middle_stream(n, pmtu=1024)
        host = buffer(ref)
        got = icrc_amd.compute_icrc_batch(host, off, lens)
        np.testing.assert_array_equal(got, oracle_icrcs(ref, off, lens))


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


# ---- fused send packetizer (icrc_write_packetize_device) vs the oracle's send path ----------
def run_packetize(engine, src: np.ndarray, msgs: np.ndarray, wire_bytes: int, fill: int = 0):
    import icrc_amd

    npk = int(msgs["npackets"].sum())
    d_src = dev(src)
    d_msgs = dev(msgs.view(np.uint8))
    d_wire = torch.full((wire_bytes,), fill, dtype=torch.uint8, device="cuda")
    d_len = torch.full((npk,), -1, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
    engine.packetize(d_src.data_ptr(), src.size, d_msgs.data_ptr(), len(msgs), npk, d_wire.data_ptr(),
                     wire_bytes, d_len.data_ptr(), d_icrc.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    return (d_wire.cpu().numpy(), d_len.cpu().numpy().view(np.uint32), d_icrc.cpu().numpy().view(np.uint32))


def _random_specs(rng, nmsg, aligned=True):
    specs, off = [], 0
    for i in range(nmsg):
        pmtu = int(rng.choice([256, 512, 1024, 2048, 4096]))
        ln = int(rng.choice([0, 1, 3, 4, 255, 256, 257, pmtu, pmtu + 1, 3 * pmtu + 7,
                             int(rng.integers(0, 20000))]))
        lva = int(rng.integers(0, 1 << 47))
        if aligned:
            off = (off + 3) & ~3
            lva &= ~3
        specs.append(dict(local_va=lva, remote_va=int(rng.integers(0, 1 << 64, dtype=np.uint64)),
                          payload_offset=off, total_len=ln, pmtu=pmtu, rkey=int(rng.integers(0, 1 << 32)),
                          dqpn=int(rng.integers(0, 1 << 24)), psn=int(rng.integers(0, 1 << 24)),
                          msn=int(rng.integers(0, 1 << 16)), dst_ip=int(rng.integers(0, 1 << 32)),
                          kind=int(rng.choice([0, 0, 1, 1, 2])), ip_id=int(rng.integers(0, 1 << 16)),
                          flags=int(rng.integers(0, 16)), lkey=int(rng.integers(0, 1 << 32)),
                          reth_len=int(rng.integers(0, 1 << 32))))
        off += ln + int(rng.integers(0, 8))
    return specs, off


@pytest.mark.parametrize("layout", ["aligned", "mixed", "odd_slots"])
def test_packetize_matches_oracle(engine, layout):
    """aligned: every packet on the word path; mixed: payloads at odd offsets (word path and
    byte path interleaved in one wave); odd_slots: every slot misaligned (byte path)."""
    import icrc_amd

    rng = np.random.default_rng({"aligned": 21, "mixed": 22, "odd_slots": 23}[layout])
    specs, src_bytes = _random_specs(rng, 40, layout == "aligned")
    msgs = icrc_amd.write_messages(specs, slot_stride=4163 if layout == "odd_slots" else 0)
    if layout == "odd_slots":
        msgs["out_offset"] += 1
    src = rng.integers(0, 256, src_bytes + 16, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1]) + 64
    want, wl, wi = oracle.send_messages(src, msgs, wire_bytes)
    got, gl, gi = run_packetize(engine, src, msgs, wire_bytes)
    np.testing.assert_array_equal(gl, wl)
    np.testing.assert_array_equal(gi, wi)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("aligned", [True, False])
def test_packetize_udp_payload_only(engine, aligned):
    """ICRC_WRITE_UDP_PAYLOAD_ONLY: every slot holds the oracle's packet from byte 28 (BTH .. ICRC,
    generate_payload_from_msg's return value, net/util.rs:183-185), pkt_len = L - 28, same ICRC;
    word path and byte path (misaligned payloads)."""
    import icrc_amd

    rng = np.random.default_rng(41 if aligned else 42)
    specs, src_bytes = _random_specs(rng, 40, aligned)
    for s in specs:
        s["flags"] = (s["flags"] & 0x0F) | icrc_amd.WRITE_UDP_PAYLOAD_ONLY
    msgs = icrc_amd.write_messages(specs)
    src = rng.integers(0, 256, src_bytes + 16, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1]) + 64
    want, wl, wi = oracle.send_messages(src, msgs, wire_bytes)
    got, gl, gi = run_packetize(engine, src, msgs, wire_bytes, fill=0xEE)
    np.testing.assert_array_equal(gi, wi)
    np.testing.assert_array_equal(gl, np.where(wl > 0, wl - 28, 0))
    k = 0
    for m in msgs:
        for s in range(int(m["npackets"])):
            o, L = int(m["out_offset"]) + s * int(m["slot_stride"]), int(wl[k])
            if L:
                np.testing.assert_array_equal(got[o: o + L - 28], want[o + 28: o + L])
                assert np.all(got[o + L - 28: o + int(m["slot_stride"])][:28] == 0xEE)
            k += 1


def test_packetize_reference_write_path(engine):
    """C3: one 20000-byte WRITE from local_va 0x..100 equals oracle.synth_write."""
    import icrc_amd

    total, pmtu, lva = 20000, 4096, 0x7F7E8EE00100
    ref, off, lens = oracle.synth_write(total, pmtu, local_va=lva, remote_va=0x7F7E8FC00000, rkey=0x2000003,
                                        dqpn=2, psn0=0, msn=0, dst_ip=0xC0A80003, payload_key=0xABCDEF)
    src = np.array([(oracle.mix64(0xABCDEF + (q >> 3)) >> (8 * (q & 7))) & 0xFF for q in range(total)],
                   dtype=np.uint8)
    stride = int(off[1] - off[0])
    msgs = icrc_amd.write_messages([dict(local_va=lva, remote_va=0x7F7E8FC00000, payload_offset=0,
                                         total_len=total, pmtu=pmtu, rkey=0x2000003, dqpn=2, psn=0, msn=0,
                                         dst_ip=0xC0A80003, kind=0)], slot_stride=stride)
    got, gl, gi = run_packetize(engine, src, msgs, ref.size)
    np.testing.assert_array_equal(gl, lens)
    for i in range(len(lens)):
        np.testing.assert_array_equal(got[int(off[i]): int(off[i]) + int(lens[i])],
                                      ref[int(off[i]): int(off[i]) + int(lens[i])])


def test_packetize_bounds(engine):
    """Packets whose slot runs past wire_bytes, or whose payload runs past d_src, are not written
    and report length 0; nothing outside the wire buffer changes."""
    import icrc_amd

    rng = np.random.default_rng(3)
    msgs = icrc_amd.write_messages([dict(local_va=0, remote_va=0, payload_offset=0, total_len=4 * 4096,
                                         pmtu=4096, rkey=1, dqpn=1, psn=0, msn=0, dst_ip=1, kind=0)])
    stride = int(msgs["slot_stride"][0])
    src = rng.integers(0, 256, 4 * 4096, dtype=np.uint8)
    wire_bytes = 3 * stride + 100  # the 4th packet does not fit
    want, wl, wi = oracle.send_messages(src, msgs, 4 * stride)
    got, gl, gi = run_packetize(engine, src, msgs, wire_bytes, fill=0xAB)
    assert gl.tolist()[:3] == wl.tolist()[:3] and gl[3] == 0 and gi[3] == 0
    for i in range(3):
        np.testing.assert_array_equal(got[i * stride: i * stride + int(wl[i])], want[i * stride: i * stride + int(wl[i])])
    assert np.all(got[3 * stride:] == 0xAB)
    # payload short by one byte: the last packet is refused, earlier ones are exact
    got, gl, gi = run_packetize(engine, src[:-1].copy(), msgs, 4 * stride)
    assert gl.tolist()[:3] == wl.tolist()[:3] and gl[3] == 0


def test_packetize_full_message_roundtrip(engine):
    """A 64 MiB READ RESPONSE at 4 KiB MTU (16384 packets): every packet verifies on the GPU,
    and a sample of packets equals the oracle's bytes."""
    import icrc_amd

    total, pmtu = 64 << 20, 4096
    rng = np.random.default_rng(9)
    msgs = icrc_amd.write_messages([dict(local_va=0x10000, remote_va=0x7F0000000000, payload_offset=0,
                                         total_len=total, pmtu=pmtu, rkey=5, dqpn=6, psn=0xFFFF00, msn=2,
                                         dst_ip=0xC0A80003, kind=1)])
    npk = int(msgs["npackets"][0])
    stride = int(msgs["slot_stride"][0])
    src = rng.integers(0, 256, total, dtype=np.uint8)
    d_src = dev(src)
    d_msgs = dev(msgs.view(np.uint8))
    d_wire = torch.zeros(npk * stride, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    engine.packetize(d_src.data_ptr(), total, d_msgs.data_ptr(), 1, npk, d_wire.data_ptr(), npk * stride,
                     d_len.data_ptr(), 0, stream=stream_handle())
    d_ok = torch.zeros(npk, dtype=torch.uint8, device="cuda")
    d_off = torch.arange(npk, dtype=torch.int64, device="cuda") * stride
    engine.verify_batch(d_wire.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), npk, d_ok.data_ptr(),
                        stream=stream_handle())
    torch.cuda.synchronize()
    assert int(d_ok.sum()) == npk
    lens = d_len.cpu().numpy()
    assert np.all(lens == 56 + pmtu + 4)
    wire = d_wire.cpu().numpy()
    sample = [0, 1, npk // 2, npk - 1]
    sub = msgs.copy()
    want, wl, _ = oracle.send_messages(src, sub, npk * stride)
    for i in sample:
        np.testing.assert_array_equal(wire[i * stride: i * stride + lens[i]], want[i * stride: i * stride + lens[i]])


# ---- fused receive (icrc_rx_parse_device) vs the oracle's is_icrc_valid + to_rdma_message -----
def run_rx(engine, buf: np.ndarray, off, lens, zero_trailer=False):
    import icrc_amd

    n = len(lens)
    d_buf = dev(buf)
    d_off = dev(np.asarray(off, np.uint64))
    d_len = dev(np.asarray(lens, np.uint32))
    d_desc = torch.zeros(n * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    d_nerr = torch.zeros(1, dtype=torch.int32, device="cuda")
    engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(), d_ok.data_ptr(),
                    zero_trailer=zero_trailer, d_nerr=d_nerr.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    desc = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    return desc, d_ok.cpu().numpy(), int(d_nerr.item()), d_buf.cpu().numpy()


def assert_desc_equal(got, want):
    for f in want.dtype.names:
        if f == "_pad":
            continue
        np.testing.assert_array_equal(got[f], want[f], err_msg=f)


@pytest.mark.parametrize("rx_variant", [-1, 16, 301])  # default (a small batch: one fused pass), two passes, per-packet stores
@pytest.mark.parametrize("layout", ["packed", "aligned"])
@pytest.mark.parametrize("zero_trailer", [False, True])
def test_rx_parse_matches_oracle(engine, layout, zero_trailer, rx_variant):
    """Every opcode x pad, corrupted opcode / transport / length / ICRC; packed offsets put most
    packets on the byte-wise path, aligned ones on the row stream.  rx_variant: the default receive
    path (verify dispatch, then descriptors from the header words) and the fused single-pass kernel
    (301: S = 2 chains, 302: S = 1, two sets in flight)."""
    import rx_cases

    engine.set_variant(rx_variant)
    try:
        _rx_parse_case(engine, layout, zero_trailer, rx_cases)
    finally:
        engine.set_variant(-1)


def _rx_parse_case(engine, layout, zero_trailer, rx_cases):
    rng = np.random.default_rng(7)
    pkts = rx_cases.make_packets(rng)
    sizes = [p.size for p in pkts]
    slot = [(s + 3) & ~3 if layout == "aligned" else s for s in sizes]
    off = np.cumsum([0] + slot[:-1]).astype(np.uint64)
    buf = np.zeros(int(off[-1]) + slot[-1] + 8, np.uint8)
    for o, p in zip(off, pkts):
        buf[int(o): int(o) + p.size] = p
    ref = buf.copy()
    want = oracle.rx_parse(ref, off, sizes, zero_trailer=zero_trailer)
    got, ok, nerr, after = run_rx(engine, buf, off, sizes, zero_trailer)
    assert_desc_equal(got, want)
    np.testing.assert_array_equal(ok, want["icrc_ok"])
    assert nerr == int(np.sum(np.asarray(sizes) < 44))
    np.testing.assert_array_equal(after, ref)


@pytest.mark.parametrize("extra", [0, 1])
@pytest.mark.parametrize("zero_trailer", [False, True])
def test_rx_parse_small_batch_boundary(engine, extra, zero_trailer):
    """The default receive takes batches of at most one packet per wave in ONE fused pass
    (descriptors collected per 64-packet block) and larger ones in two passes: both sides of the
    boundary (#CUs x 16 packets, and one more), a 16 MiB WRITE's packets with mixed lengths and
    misaligned ones, one flipped bit per 97 packets."""
    import icrc_amd

    n = torch.cuda.get_device_properties(0).multi_processor_count * 16 + extra
    rng = np.random.default_rng(11 + extra)
    buf, off, lens = oracle.synth_middle_stream(n, psn0=0x10)
    # ragged: some packets shortened to other MTU classes / odd lengths (pad), a few misaligned
    pkts = [buf[int(o): int(o) + int(L)].copy() for o, L in zip(off, lens)]
    for i in rng.choice(n, n // 8, replace=False):
        L = int(rng.choice([60, 61, 316, 1084, 2001]))
        p = pkts[i][:L].copy()
        p[2:4] = np.frombuffer(int(L).to_bytes(2, "big"), np.uint8)
        pkts[i] = p
    sizes = np.array([p.size for p in pkts], np.uint32)
    gaps = rng.integers(0, 4, n) * (rng.random(n) < 0.05)  # 5 % start off a word boundary
    offs = np.zeros(n, np.uint64)
    pos = 0
    for i, p in enumerate(pkts):
        pos += int(gaps[i])
        offs[i] = pos
        pos += p.size
    b = np.zeros(pos + 8, np.uint8)
    for o, p in zip(offs, pkts):
        b[int(o): int(o) + p.size] = p
    for i in range(0, n, 97):
        b[int(offs[i]) + 50] ^= 0x01
    ref = b.copy()
    want = oracle.rx_parse(ref, offs, sizes, zero_trailer=zero_trailer)
    got, ok, nerr, after = run_rx(engine, b, offs, sizes, zero_trailer)
    assert_desc_equal(got, want)
    np.testing.assert_array_equal(ok, want["icrc_ok"])
    np.testing.assert_array_equal(after, ref)
    assert icrc_amd.RX_DESC_DTYPE.itemsize == 72


@pytest.mark.parametrize("ragged", [False, True])
@pytest.mark.parametrize("rx_variant", [-1, 301, 302])
def test_rx_parse_c1_stream(engine, ragged, rx_variant):
    """A 4 KiB WRITE_MIDDLE stream (strided, or the same packets through offset / length arrays) with
    one flipped bit per 1024; the ok bytes go to d_ok as well.  70 000 packets: every wave of the
    grid owns whole 64-packet blocks."""
    import icrc_amd

    n = 70000
    buf, off, lens = oracle.synth_middle_stream(n, psn0=0xFFFF00)
    L = int(lens[0])
    for i in range(0, n, 1024):
        buf[int(off[i]) + 200] ^= 0x10
    want = oracle.rx_parse(buf.copy(), off, lens)
    d_buf = dev(buf)
    d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    engine.set_variant(rx_variant)
    try:
        if ragged:
            d_off, d_len = dev(np.asarray(off, np.uint64)), dev(np.asarray(lens, np.uint32))
            engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(),
                            d_ok.data_ptr(), stream=stream_handle())
        else:
            engine.rx_parse(d_buf.data_ptr(), 0, 0, n, d_desc.data_ptr(), d_ok.data_ptr(), stride=L, length=L,
                            stream=stream_handle())
        torch.cuda.synchronize()
    finally:
        engine.set_variant(-1)
    got = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    assert_desc_equal(got, want)
    np.testing.assert_array_equal(d_ok.cpu().numpy(), got["icrc_ok"])
    assert int(np.sum(got["icrc_ok"] == 0)) == (n + 1023) // 1024
    assert np.all(got["payload_len"] == 4096) and np.all(got["status"] == 0)


def _strided_rx_batch(L, n, stride, seed):
    """n packets of exactly L bytes at `stride`: the header bytes of rx_cases' corpus (every opcode,
    the corrupted opcode / transport / pad ones) round-robin, random bytes after them, the ICRC
    written into each trailer, then every 29th trailer flipped."""
    import rx_cases

    rng = np.random.default_rng(seed)
    corpus = [p for p in rx_cases.make_packets(rng) if p.size >= 44]
    buf = rng.integers(0, 256, n * stride + 8, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    lens = np.full(n, L, np.uint32)
    for i in range(n):
        t = corpus[i % len(corpus)]
        m = min(L - 4, t.size - 4)
        buf[i * stride: i * stride + m] = t[:m]
    ic = oracle.compute_icrc_batch(buf, off, lens)
    tr = (off + np.uint64(L - 4)).astype(np.int64)
    for k in range(4):
        buf[tr + k] = ((ic >> (8 * k)) & 0xFF).astype(np.uint8)
    buf[tr[::29]] ^= 0x40
    return buf, off, lens


@pytest.mark.parametrize("L", [44, 48, 60, 64, 72, 76, 316, 320, 652, 1084, 1088])
@pytest.mark.parametrize("zero_trailer", [False, True])
def test_rx_parse_strided_short_one_pass(engine, L, zero_trailer):
    """Strided batches of short packets take ONE pass (icrc_oct_rx_kernel: the oct verify keeps
    the header words it loads, words 7..17, and stores the descriptors itself): every opcode's
    header and the corrupted ones at lengths from 44 B (the trailer inside word 10) to the oct
    kernel's 1088, a batch above the one-pass small-batch boundary with a ragged last block, packed
    and padded strides; descriptors, ok bytes and the zeroed trailers against the oracle, and the
    same descriptors with no ok array."""
    import icrc_amd

    n = torch.cuda.get_device_properties(0).multi_processor_count * 16 * 3 + 37
    stride = L if L % 8 else L + 12
    buf, off, lens = _strided_rx_batch(L, n, stride, L * 2 + int(zero_trailer))
    ref = buf.copy()
    want = oracle.rx_parse(ref, off, lens, zero_trailer=zero_trailer)
    for with_ok in (True, False):
        d_buf = dev(buf)
        d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
        d_ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        engine.rx_parse(d_buf.data_ptr(), 0, 0, n, d_desc.data_ptr(), d_ok.data_ptr() if with_ok else 0,
                        zero_trailer=zero_trailer, stride=stride, length=L, stream=stream_handle())
        torch.cuda.synchronize()
        got = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
        assert_desc_equal(got, want)
        if with_ok:
            np.testing.assert_array_equal(d_ok.cpu().numpy(), want["icrc_ok"])
        np.testing.assert_array_equal(d_buf.cpu().numpy(), ref)
    assert int(np.sum(want["icrc_ok"] == 0)) >= (n + 28) // 29  # the flipped trailers (and the corpus' own)
    assert len(set(want["status"].tolist())) >= 3  # ok, invalid opcode / transport, truncated
    assert L < 76 or len(set(want["opcode"].tolist())) >= 12


@pytest.mark.parametrize("L", [316, 1084])
def test_rx_parse_strided_short_one_pass_full_blocks(engine, L):
    """The one-pass receive over 300 000 packets: every wave owns whole 64-packet blocks (several
    per wave, the per-wave LDS record reused block after block)."""
    import icrc_amd

    n = 300_000
    buf, off, lens = _strided_rx_batch(L, n, L, 5 + L)
    want = oracle.rx_parse(buf.copy(), off, lens)
    d_buf = dev(buf)
    d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.rx_parse(d_buf.data_ptr(), 0, 0, n, d_desc.data_ptr(), d_ok.data_ptr(), stride=L, length=L,
                    stream=stream_handle())
    torch.cuda.synchronize()
    got = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    assert_desc_equal(got, want)
    np.testing.assert_array_equal(d_ok.cpu().numpy(), want["icrc_ok"])


@pytest.mark.parametrize("zero_trailer", [False, True])
def test_rx_parse_ragged_one_pass(engine, zero_trailer):
    """Ragged batches with more than 32 packets per wave take ONE launch (icrc_hybrid_rx_kernel):
    the one-pass receive on the oct kernel's packets, then long_body's verify and a sweep for the
    rest.  Mostly 316-B packets with 1084 / 1088 / 1089 / 4156 / 2001-B ones, short (44, 48, 60)
    and odd-length (61) ones, 3 % starting off a word boundary, one flipped ICRC per 29 packets;
    descriptors, ok bytes and trailers against the oracle, and the descriptors with no ok array."""
    import icrc_amd
    import rx_cases

    rng = np.random.default_rng(31 + int(zero_trailer))
    n = torch.cuda.get_device_properties(0).multi_processor_count * 16 * 32 + 5003
    corpus = [p for p in rx_cases.make_packets(rng) if p.size >= 44]
    lens = rng.choice([316, 1084, 1088, 1089, 4156, 2001, 44, 48, 60, 61], n,
                      p=[0.80, 0.05, 0.02, 0.02, 0.05, 0.02, 0.01, 0.01, 0.01, 0.01]).astype(np.uint32)
    gaps = rng.integers(1, 4, n) * (rng.random(n) < 0.03)
    off = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += int(lens[i])
    buf = rng.integers(0, 256, pos + 8, dtype=np.uint8)
    for i in range(n):
        t = corpus[i % len(corpus)]
        m = min(int(lens[i]) - 4, t.size - 4)
        buf[int(off[i]): int(off[i]) + m] = t[:m]
    ic = oracle.compute_icrc_batch(buf, off, lens)
    tr = (off + lens - 4).astype(np.int64)
    for k in range(4):
        buf[tr + k] = ((ic >> (8 * k)) & 0xFF).astype(np.uint8)
    buf[tr[::29]] ^= 0x40
    ref = buf.copy()
    want = oracle.rx_parse(ref, off, lens, zero_trailer=zero_trailer)
    for with_ok in (True, False):
        d_buf = dev(buf)
        d_off, d_len = dev(off), dev(lens)
        d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
        d_ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        d_nerr = torch.zeros(1, dtype=torch.int32, device="cuda")
        engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(),
                        d_ok.data_ptr() if with_ok else 0, zero_trailer=zero_trailer, d_nerr=d_nerr.data_ptr(),
                        stream=stream_handle())
        torch.cuda.synchronize()
        got = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
        assert_desc_equal(got, want)
        if with_ok:
            np.testing.assert_array_equal(d_ok.cpu().numpy(), want["icrc_ok"])
        np.testing.assert_array_equal(d_buf.cpu().numpy(), ref)
    assert int(np.sum(want["status"] == 0)) > n // 2 and int(np.sum(want["icrc_ok"] == 0)) >= n // 29


def test_rx_parse_mixed_mtu_stream_full(engine):
    """the receive parse on the emulator's mixed-MTU batch itself (configs[2]'s
    generator, mixed_mtu_stream: 256 B / 1 KiB / 4 KiB MTU classes, power law, 10 % ragged LAST
    packets) at 1 Mi packets — the default ragged dispatch (the one-pass ragged ring, the long-packet
    verify and the sweep) against the oracle, every descriptor and ok byte, with one flipped ICRC per
    97 packets; then the same batch with zero_trailer."""
    import icrc_amd
    from icrc_amd import workloads

    wm = workloads.mixed_mtu_stream(1 << 20, seed=77)
    s = stream_handle()
    d_buf = workloads.synthesize(engine, wm, stream=s)
    torch.cuda.synchronize()
    buf = d_buf.cpu().numpy()
    del d_buf
    off, lens = np.ascontiguousarray(wm.off, np.uint64), np.ascontiguousarray(wm.lens, np.uint32)
    ic = oracle.compute_icrc_batch(buf, off, lens)
    tr = (off + lens - 4).astype(np.int64)
    for k in range(4):
        buf[tr + k] = ((ic >> (8 * k)) & 0xFF).astype(np.uint8)
    buf[tr[::97]] ^= 0x08
    for zero_trailer in (False, True):
        ref = buf.copy()
        want = oracle.rx_parse(ref, off, lens, zero_trailer=zero_trailer)
        d_buf = dev(buf)
        d_off, d_len = dev(off), dev(lens)
        d_desc = torch.zeros(wm.n * 72, dtype=torch.uint8, device="cuda")
        d_ok = torch.full((wm.n,), 7, dtype=torch.uint8, device="cuda")
        engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n, d_desc.data_ptr(), d_ok.data_ptr(),
                        zero_trailer=zero_trailer, stream=s)
        torch.cuda.synchronize()
        got = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
        assert_desc_equal(got, want)
        np.testing.assert_array_equal(d_ok.cpu().numpy(), want["icrc_ok"])
        if zero_trailer:
            np.testing.assert_array_equal(d_buf.cpu().numpy(), ref)
        del d_buf, d_off, d_len, d_desc, d_ok
    assert int(np.sum(want["icrc_ok"] == 0)) == (wm.n + 96) // 97
    assert np.all(want["status"] == 0)
    assert len(set(want["payload_len"].tolist())) > 100  # the ragged LAST packets' lengths


@pytest.mark.parametrize("zero_trailer", [False, True])
def test_rx_parse_dense_and_sparse_long_ranges(engine, zero_trailer):
    """The ragged receive's two descriptor paths for long packets in one batch: a first region of
    4156-B packets (waves walking it take the dense C1 ring, raise the sweep's second flag and leave
    every long packet's descriptor to the sweep), then a region of 316-B packets with one 4156-B or
    2001-B packet per ~60 (waves there take the sparse walk and write their long packets'
    descriptors themselves; the sweep rewrites them with the same bytes).  Every descriptor, ok
    byte and trailer against the oracle."""
    import icrc_amd

    rng = np.random.default_rng(4242 + int(zero_trailer))
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    n_dense = n_cu * 16 * 64 // 4  # about a quarter of the grid's waves on all-long ranges
    n_sparse = n_cu * 16 * 64 * 3 // 4
    lens = np.concatenate([np.full(n_dense, 4156, np.uint32),
                           np.where(rng.random(n_sparse) < 1 / 60, rng.choice([4156, 2001], n_sparse), 316)
                           .astype(np.uint32)])
    n = lens.size
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(((lens[:-1].astype(np.uint64) + 3) // 4) * 4)
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    # BTH of an RC WRITE_MIDDLE (opcode 0x07, transport RC, pad 0) on every packet: most parse OK
    buf[off.astype(np.int64) + 28] = 0x07
    buf[off.astype(np.int64) + 29] = 0x00
    ic = oracle.compute_icrc_batch(buf, off, lens)
    tr = (off + lens - 4).astype(np.int64)
    for k in range(4):
        buf[tr + k] = ((ic >> (8 * k)) & 0xFF).astype(np.uint8)
    buf[tr[::53]] ^= 0x04
    ref = buf.copy()
    want = oracle.rx_parse(ref, off, lens, zero_trailer=zero_trailer)
    d_buf = dev(buf)
    d_off, d_len = dev(off), dev(lens)
    d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(), d_ok.data_ptr(),
                    zero_trailer=zero_trailer, stream=stream_handle())
    torch.cuda.synchronize()
    got = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    assert_desc_equal(got, want)
    np.testing.assert_array_equal(d_ok.cpu().numpy(), want["icrc_ok"])
    np.testing.assert_array_equal(d_buf.cpu().numpy(), ref)
    assert int(np.sum(want["icrc_ok"] == 0)) >= n // 53 and int(np.sum(want["status"] == 0)) > n // 2


def test_send_receive_roundtrip(engine):
    """Packetize 24 WRITE / READ RESPONSE messages on the GPU, parse them on the GPU, and place each
    payload at its RETH va: the memory region equals the source bytes (C3 closed on-device)."""
    import icrc_amd

    rng = np.random.default_rng(31)
    specs, src_bytes = _random_specs(rng, 24, True)
    region = 1 << 20
    for k, s in enumerate(specs):  # remote va = payload position inside a 1 MiB region at 0x10000000
        s["remote_va"] = 0x10000000 + s["payload_offset"]
    assert src_bytes < region
    msgs = icrc_amd.write_messages(specs)
    src = rng.integers(0, 256, region, dtype=np.uint8)
    npk = int(msgs["npackets"].sum())
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1])
    wire, plen, picrc = run_packetize(engine, src, msgs, wire_bytes)
    off = np.concatenate([int(m["out_offset"]) + np.arange(int(m["npackets"]), dtype=np.uint64) * int(m["slot_stride"])
                          for m in msgs]).astype(np.uint64)
    desc, ok, nerr, _ = run_rx(engine, wire, off, plen)
    assert nerr == 0 and np.all(ok == 1) and np.all(desc["status"] == 0)
    mr = np.zeros(region, np.uint8)
    for d in desc:
        if d["opcode"] == 0x0C:
            assert d["payload_len"] == 0 and d["flags"] & icrc_amd.RX_HAS_SECONDARY_RETH
            continue
        o, ln, va = int(d["payload_offset"]), int(d["payload_len"]), int(d["reth_va"])
        mr[va - 0x10000000: va - 0x10000000 + ln] = wire[o: o + ln]
    for s in specs:
        if s["kind"] == 2:  # a read request carries no payload (its total_len is the local SGE's)
            continue
        a, ln = s["payload_offset"], s["total_len"]
        np.testing.assert_array_equal(mr[a: a + ln], src[a: a + ln])


# ---- batched IPv4 header checksum (icrc_ipv4_checksum_device) -------------------------------
def test_ipv4_checksum_reference_vectors_and_fill(engine):
    """responser.rs:370-393 vectors (checksum over the stored header), then fill mode on random
    headers at odd offsets: the stored checksum equals the oracle's and re-summing gives 0."""
    from golden_kats import IPV4_HEADERS

    rng = np.random.default_rng(12)
    hdrs = [np.frombuffer(h, np.uint8) for h, _ in IPV4_HEADERS]
    hdrs += [rng.integers(0, 256, 20, dtype=np.uint8) for _ in range(500)]
    off = np.cumsum([0] + [21] * (len(hdrs) - 1)).astype(np.uint64)  # odd offsets: byte path
    buf = np.zeros(int(off[-1]) + 21, np.uint8)
    for o, h in zip(off, hdrs):
        buf[int(o): int(o) + 20] = h
    zeroed = [h.copy() for h in hdrs]
    for z in zeroed:
        z[10:12] = 0
    n = len(hdrs)
    d_buf, d_off = dev(buf), dev(off)
    d_c = torch.zeros(n, dtype=torch.int16, device="cuda")
    engine.ipv4_checksum(d_buf.data_ptr(), n, d_off=d_off.data_ptr(), d_csum=d_c.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    raw = d_c.cpu().numpy().view(np.uint16)
    assert [int(x) for x in raw] == [oracle.ipv4_checksum(h) for h in hdrs]
    for (h, want), got in zip(IPV4_HEADERS, raw):
        assert int(got) == want
    engine.ipv4_checksum(d_buf.data_ptr(), n, d_off=d_off.data_ptr(), d_csum=d_c.data_ptr(), fill=True,
                         stream=stream_handle())
    torch.cuda.synchronize()
    filled = d_buf.cpu().numpy()
    got = d_c.cpu().numpy().view(np.uint16)
    for i, (o, z) in enumerate(zip(off, zeroed)):
        c = oracle.ipv4_checksum(z)
        assert int(got[i]) == c
        h = filled[int(o): int(o) + 20]
        assert (int(h[10]) << 8 | int(h[11])) == c and oracle.ipv4_checksum(h) == 0


@pytest.mark.parametrize("variant", [-1, 140])
def test_ragged_offsets_beyond_2GiB(engine, variant):
    """Offset arrays with entries >= 2^31 and >= 2^32 (v_readlane returns int: widening it must not
    sign-extend): compute, verify and receive-parse against the oracle.  Variant 140 forces the
    hybrid dispatch, so the oct kernel sees blocks whose packets lie 2 GiB apart (outside its
    [-1 GiB, +1 GiB) block window: the per-packet path)."""
    import icrc_amd

    engine.set_variant(variant)
    try:
        _offsets_beyond_2gib(engine, icrc_amd)
    finally:
        engine.set_variant(-1)


def _offsets_beyond_2gib(engine, icrc_amd):

    rng = np.random.default_rng(44)
    pkts, _ = [], None
    for i in range(300):
        L = int(rng.choice([44, 316, 1084, 4156, 4157, 777]))
        pkts.append(rng.integers(0, 256, L, dtype=np.uint8))
    total = (1 << 32) + (1 << 20)
    d_buf = torch.zeros(total, dtype=torch.uint8, device="cuda")
    starts = [(1 << 31) - 5000, (1 << 32) - 3000]
    off, pos = [], 0
    for i, p in enumerate(pkts):
        base = starts[i % 2] + (i // 2) * 4200
        off.append(base)
        d_buf[base: base + p.size] = torch.from_numpy(p).cuda()
    off = np.asarray(off, np.uint64)
    lens = np.asarray([p.size for p in pkts], np.uint32)
    d_off, d_len = dev(off), dev(lens)
    n = len(pkts)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(), True, 0,
                         stream_handle())
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(), False, 0,
                        stream_handle())
    d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
    engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    want = [oracle.compute_icrc(p) for p in pkts]
    assert [int(x) for x in d_out.cpu().numpy().view(np.uint32)] == want
    assert d_ok.cpu().numpy().tolist() == [1] * n
    desc = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    assert np.all(desc["icrc_ok"] == 1)
    ok_parse = desc["status"] == 0
    assert np.all(desc["payload_offset"][ok_parse] >= np.asarray(off)[ok_parse] + 28)
    del d_buf
    torch.cuda.empty_cache()


def test_ragged_dense_long_walk_across_4GiB(engine):
    """The hybrid launch's dense long-packet walk (scalar (offset, length) loads one set ahead, the
    waves' age skew) on 12 288 packets of 4156 B whose offsets cross 2^32: compute with trailers,
    verify against the oracle, then verify with a flipped bit every 97 packets."""
    rng = np.random.default_rng(4097)
    n, L = 12288, 4156
    base = (1 << 32) - 6 * 1024 * L  # a quarter of the packets below 4 GiB, the rest above
    total = base + n * L + 64
    d_buf = torch.zeros(total, dtype=torch.uint8, device="cuda")
    pk = rng.integers(0, 256, n * L, dtype=np.uint8)
    d_buf[base: base + n * L] = torch.from_numpy(pk).cuda()
    off = base + np.arange(n, dtype=np.uint64) * np.uint64(L)
    lens = np.full(n, L, np.uint32)
    d_off, d_len = dev(off), dev(lens)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(), True, 0,
                         stream_handle())
    torch.cuda.synchronize()
    rel = np.arange(n, dtype=np.uint64) * np.uint64(L)
    want = oracle_icrcs(pk, rel, lens)
    np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), want)
    bad = np.arange(0, n, 97)
    for i in bad:
        d_buf[int(off[i]) + 100] ^= 0x01
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(), False, 0,
                        stream_handle())
    torch.cuda.synchronize()
    expect = np.ones(n, np.uint8)
    expect[bad] = 0
    np.testing.assert_array_equal(d_ok.cpu().numpy(), expect)
    del d_buf
    torch.cuda.empty_cache()


def test_empty_batches_are_noops(engine):
    """n == 0 on every device entry point: OK, nothing written (the reference's loops simply do
    not run on an empty packet list)."""
    import icrc_amd

    guard = torch.full((64,), 0x5A, dtype=torch.uint8, device="cuda")
    p = guard.data_ptr()
    s = stream_handle()
    engine.compute_batch(p, p, p, 0, p, write_trailer=True, stream=s)
    engine.verify_batch(p, p, p, 0, p, zero_trailer=True, stream=s)
    engine.compute_strided(p, 64, 64, 0, p, True, s)
    engine.verify_strided(p, 64, 64, 0, p, True, s)
    engine.rx_parse(p, 0, 0, 0, p, p, stride=64, length=64, stream=s)
    engine.ipv4_checksum(p, 0, stride=64, d_csum=p, fill=True, stream=s)
    torch.cuda.synchronize()
    assert bool((guard == 0x5A).all().item())
    assert icrc_amd.compute_icrc_batch(np.zeros(0, np.uint8), [], []).size == 0


@pytest.mark.parametrize("variant", [-1, 40, 140])
@pytest.mark.parametrize("pmtu", [256, 1024])
def test_short_strided_stream_oct_path(engine, pmtu, variant):
    """Uniform strided batches of short packets (at this size the one-packet pipeline by default;
    forced to the oct kernel, 40, or the forced split, 140): compute, trailer write and verify
    against the oracle."""
    n = 2000 + pmtu // 256  # not a multiple of 4 or 64
    buf, off, lens = oracle.synth_middle_stream(n, pmtu=pmtu)
    L = int(lens[0])
    d = dev(buf)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.set_variant(variant)
    try:
        engine.compute_strided(d.data_ptr(), L, L, n, d_out.data_ptr(), True, stream_handle())
        torch.cuda.synchronize()
    finally:
        engine.set_variant(-1)
    want = oracle_icrcs(buf, off, lens)
    np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), want)
    host = d.cpu().numpy()
    np.testing.assert_array_equal(host.reshape(n, L)[:, L - 4:].copy().view(np.uint32).ravel(), want)
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.set_variant(variant)
    try:
        engine.verify_strided(d.data_ptr(), L, L, n, d_ok.data_ptr(), False, stream_handle())
        torch.cuda.synchronize()
    finally:
        engine.set_variant(-1)
    assert bool((d_ok == 1).all().item())


@pytest.mark.parametrize("variant", [-1, 40, 140, 240])
@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_tiny_batches_every_path(engine, n, variant):
    """1-5 packets: every wave but a few idle, sets of eight partly empty, chunks below one block;
    the default (one-packet pipeline at this size), the oct kernel (40) and the split forced (140,
    240)."""
    rng = np.random.default_rng(900 + n)
    lens = rng.choice([44, 316, 1084, 4156, 9000], n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]), dtype=np.uint8)
    engine.set_variant(variant)
    try:
        out, nerr, _ = run_batch(engine, buf, off, lens)
    finally:
        engine.set_variant(-1)
    assert nerr == 0
    np.testing.assert_array_equal(out, oracle_icrcs(buf, off, lens))


@pytest.mark.parametrize("delta", [-4095, -4063, -1, 0, 1])
def test_small_batch_grid_boundary(engine, delta):
    """The small-batch dispatch (at most one packet per wave of the full grid: two packets per wave
    on half the workgroups, round 6) at and around its bound of #CUs x 16 packets (n = #CUs x 16 +
    delta, at least 1: 1, 33, bound - 1, the bound, bound + 1 on 256 CUs): mixed lengths with short
    (error) and long packets, 3 % misaligned offsets; compute with write_trailer, then verify with
    zero_trailer, against the oracle (ICRCs, written trailers, verify results, zeroed trailers)."""
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    n = max(1, n_cu * 16 + delta)
    rng = np.random.default_rng(7100 + n)
    lens = rng.choice([40, 44, 61, 316, 1084, 1089, 4156, 9000], n, p=[.02, .05, .1, .3, .2, .03, .25, .05]).astype(np.uint32)
    gap = np.where(rng.random(n) < 0.03, rng.integers(1, 4, n), 0).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(((lens[:-1].astype(np.uint64) + 3) // 4) * 4 + gap[:-1])
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    ok_len = lens >= 44
    out, nerr, wrote = run_batch(engine, buf, off, lens, write_trailer=True)
    want = oracle_icrcs(buf, off[ok_len], lens[ok_len])
    np.testing.assert_array_equal(out[ok_len], want)
    assert nerr == int((~ok_len).sum())
    tr = (off[ok_len] + lens[ok_len] - 4).astype(np.int64)
    got_tr = wrote[tr] | (wrote[tr + 1].astype(np.uint32) << 8) | (wrote[tr + 2].astype(np.uint32) << 16) | \
        (wrote[tr + 3].astype(np.uint32) << 24)
    np.testing.assert_array_equal(got_tr, want)
    d_buf, d_off, d_len = dev(wrote), dev(off), dev(lens)
    d_ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(), True, 0, stream_handle())
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy()
    assert np.all(ok[ok_len] == 1) and np.all(ok[~ok_len] == 0xFF)
    after = d_buf.cpu().numpy()
    assert not any(after[tr + k].any() for k in range(4))


def test_oct_frame_boundaries(engine):
    """The oct kernel's frame arithmetic at its edges, through the default hybrid dispatch (a batch
    big enough to split): 1- and 2-frame packets (L = 320 / 324: 10 / 11 rows), 4 frames (1084,
    1088: 34 rows), the hand-off to the long kernel (1089, 1092), every residue of N mod 8 (the
    front padding), mixed in blocks and in runs, with trailer write, verify and zeroing."""
    rng = np.random.default_rng(1088)
    n = 12000
    choices = np.array([44, 48, 60, 316, 320, 324, 328, 644, 964, 1080, 1084, 1088, 1092, 1096, 2048, 4156])
    lens = rng.choice(choices, n).astype(np.uint32)
    lens[2000:2640] = 1088                      # whole blocks of 4-frame packets
    lens[3000:3640] = 324                       # whole blocks of 2-frame packets
    lens[5000:5640] = rng.integers(11, 273, 640) * 4  # every row count 2..34
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    want = oracle_icrcs(buf, off, lens)
    out, nerr, wrote = run_batch(engine, buf, off, lens, write_trailer=True)
    assert nerr == 0
    np.testing.assert_array_equal(out, want)
    tr = (off + lens.astype(np.uint64) - 4).astype(np.int64)[:, None] + np.arange(4)
    np.testing.assert_array_equal(wrote[tr].reshape(-1).view("<u4"), want)
    bad = np.arange(7, n, 97)
    for i in bad:  # a covered byte: payload, or the IPv4 total length of a 44-byte packet
        L = int(lens[i])
        wrote[int(off[i]) + (int(rng.integers(40, L - 4)) if L > 44 else 2)] ^= 0x80
    d_b, d_o, d_l = dev(wrote), dev(off), dev(lens)
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_b.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), n, d_ok.data_ptr(), zero_trailer=True,
                        stream=stream_handle())
    torch.cuda.synchronize()
    ok = d_ok.cpu().numpy()
    expect = np.ones(n, np.uint8)
    expect[bad] = 0
    np.testing.assert_array_equal(ok, expect)
    assert not d_b.cpu().numpy()[tr].any()


def test_split_batches_concurrent_streams(engine):
    """Split (hybrid) ragged batches issued from four host threads on four streams of one
    engine: the fork / join onto the engine's side stream must keep every caller's long-packet
    half ordered inside that caller's stream."""
    import threading

    rng = np.random.default_rng(4242)
    jobs = []
    for t in range(4):
        n = 5000 + 500 * t  # above one packet per wave of the grid: the split (fork / join) path
        lens = rng.choice([316, 1084, 4156, 9000], n, p=[0.6, 0.2, 0.15, 0.05]).astype(np.uint32)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        buf = rng.integers(0, 256, int(off[-1] + lens[-1]), dtype=np.uint8)
        jobs.append((buf, off, lens, oracle_icrcs(buf, off, lens)))
    errors = []

    def worker(t):
        try:
            buf, off, lens, want = jobs[t]
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                d_buf, d_off, d_len = dev(buf), dev(off), dev(lens)
                for _ in range(5):
                    d_out = torch.zeros(len(lens), dtype=torch.int32, device="cuda")
                    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens),
                                         d_out.data_ptr(), stream=s.cuda_stream)
                    got = d_out.cpu().numpy().view(np.uint32)  # syncs this stream only
                    if not np.array_equal(got, want):
                        errors.append(f"thread {t}: {int((got != want).sum())} mismatches")
                        return
        except Exception as exc:  # noqa: BLE001
            errors.append(f"thread {t}: {exc!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    torch.cuda.synchronize()
    assert not errors, errors


DIAGNOSTIC_VARIANTS = (15, 18, 19, 21, 22, 23, 27, 28, 29, 30, 33, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 141, 146, 148, 241)


def test_kernel_variant_validation(engine, ab_engine):
    """The product library accepts only result-exact variants; the diagnostics (wrong results by
    design) exist only in the A/B library (libicrc_amd_ab.so).  The retired quad kernels (20,
    24-26, 31, 32, 35 and their hybrid forms) are refused by both."""
    import icrc_amd

    for v in (-1, 0, 13, 16, 17, 40, 140, 240, 301, 302):
        engine.set_variant(v)
    engine.set_variant(-1)
    retired = (20, 24, 25, 26, 31, 32, 35, 120, 124, 220, 224)
    for v in (-2, 1, 10, 14, 23, 27, 36, 53, 99, 100, 116, 153, 303, 400) + DIAGNOSTIC_VARIANTS + retired:
        with pytest.raises(icrc_amd.IcrcError) as e:
            engine.set_variant(v)
        assert e.value.rc == icrc_amd.EINVAL, v
    for v in (-1, 0, 13, 16, 17, 40, 140, 240, 301, 302) + DIAGNOSTIC_VARIANTS:
        ab_engine.set_variant(v)
    ab_engine.set_variant(-1)
    for v in retired:
        with pytest.raises(icrc_amd.IcrcError):
            ab_engine.set_variant(v)
    assert "A/B build" in icrc_amd.ab_library().icrc_version().decode() and "A/B" not in icrc_amd.version()


def test_scalar_surface_accepts_any_writable_buffer():
    """is_icrc_valid on a bytearray / memoryview zeroes the caller's own trailer (no copy)."""
    import icrc_amd

    pkt = bytearray(KAT1)
    assert icrc_amd.is_icrc_valid(pkt)
    assert pkt[-4:] == b"\0\0\0\0"
    mv = memoryview(bytearray(KAT1))
    assert icrc_amd.is_icrc_valid(mv)
    assert bytes(mv[-4:]) == b"\0\0\0\0"
    assert icrc_amd.compute_icrc(bytes(KAT1)) == KAT1_ICRC  # read-only is fine for compute


def test_scalar_three_threads_parity():
    """compute_icrc / is_icrc_valid (the per-packet drop-ins, packet_processor.rs:275-301 and
    341-353) from three host threads at once: the combining submitter folds concurrent calls into
    one launch per mode; each caller must still get its own packet's answer, and is_icrc_valid must
    zero exactly the caller's trailer."""
    import threading

    import icrc_amd

    rng = np.random.default_rng(333)
    jobs = []
    for t in range(3):
        pk = []
        for _ in range(400):
            L = int(rng.choice([44, 45, 47, 60, 316, 1084, 4156, 9000, 65535]))
            pk.append(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        jobs.append(pk)
    want = [[oracle.compute_icrc(p) for p in pk] for pk in jobs]
    errors = []
    barrier = threading.Barrier(3)

    def worker(t):
        try:
            barrier.wait(timeout=60)
            for i, p in enumerate(jobs[t]):
                got = icrc_amd.compute_icrc(p)
                if got != want[t][i]:
                    errors.append(f"thread {t} compute #{i} (L={len(p)}): {got:#x} != {want[t][i]:#x}")
                    return
                good = bytearray(p[:-4]) + want[t][i].to_bytes(4, "little")
                bad = bytearray(good)
                bad[len(bad) // 2] ^= 0x10
                if not icrc_amd.is_icrc_valid(good) or bytes(good[-4:]) != b"\0\0\0\0":
                    errors.append(f"thread {t} verify #{i}: valid packet rejected or trailer kept")
                    return
                if icrc_amd.is_icrc_valid(bad):
                    errors.append(f"thread {t} verify #{i}: corrupted packet accepted")
                    return
        except Exception as exc:  # noqa: BLE001
            errors.append(f"thread {t}: {exc!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads), "scalar callers hung"
    assert not errors, errors[:5]


def test_packetize_read_requests_and_oversize(engine):
    """READ REQUEST messages (Read::handle, read.rs:33-89: one 76-byte double-RETH packet,
    opcode 0x0C) interleaved with WRITEs, and a WRITE whose pmtu makes a segment longer than an
    IPv4 packet can be (L > 65535: PacketWriter::write returns LengthTooLong,
    packet_processor.rs:226-227) — that packet reports length 0 and writes nothing."""
    import icrc_amd

    rng = np.random.default_rng(76)
    specs = []
    for i in range(24):
        if i % 3 == 2:
            specs.append(dict(local_va=int(rng.integers(0, 1 << 47)), remote_va=int(rng.integers(0, 1 << 47)),
                              total_len=int(rng.integers(0, 1 << 31)), reth_len=int(rng.integers(0, 1 << 31)),
                              pmtu=4096, rkey=int(rng.integers(0, 1 << 32)), lkey=int(rng.integers(0, 1 << 32)),
                              dqpn=i, psn=int(rng.integers(0, 1 << 24)), msn=i, dst_ip=0xC0A80003, kind=2,
                              flags=int(rng.choice([0, 8, 9, 12, 13])), ip_id=1))
        else:
            specs.append(dict(local_va=0x1000 * i, remote_va=0x7F0000000000 + 0x10000 * i, payload_offset=1024 * i,
                              total_len=int(rng.integers(1, 9000)), pmtu=4096, rkey=3, dqpn=i, psn=i, msn=i,
                              dst_ip=0xC0A80003, kind=0, ip_id=1))
    # oversize: pmtu 65536 -> a 65536-byte first segment, L = 65596 > 65535
    specs.append(dict(local_va=0, remote_va=0, payload_offset=0, total_len=70000, pmtu=65536, rkey=1, dqpn=1,
                      psn=0, msn=0, dst_ip=1, kind=0, slot_stride=70000))
    msgs = icrc_amd.write_messages(specs)
    src = rng.integers(0, 256, 80000, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1]) + 64
    want, wl, wi = oracle.send_messages(src, msgs, wire_bytes)
    got, gl, gi = run_packetize(engine, src, msgs, wire_bytes)
    rr = msgs["first_packet"][msgs["kind"] == 2]
    assert np.all(gl[rr] == 76) and np.all(wl[rr] == 76)
    big = int(msgs["first_packet"][-1])
    assert gl[big] == 0 and gi[big] == 0 and gl[big + 1] > 0  # the second segment (4464 B) fits
    np.testing.assert_array_equal(gl, wl)
    np.testing.assert_array_equal(gi, wi)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("variant", [-1, 140])
def test_hybrid_segregated_halves(engine, variant):
    """The one-launch hybrid kernel (default) and the two-kernel fork / join (140) on a ragged
    batch whose first half is all 4156-byte packets and second half all 316-byte ones: the oct
    workgroups over the first half and the long-packet workgroups over the second both exit before
    their table loads.  Compute with write_trailer, then verify with zero_trailer, against the
    oracle; one flipped bit in each half must read as a mismatch."""
    n_long, n_short = 8192, 8192
    bl, _, ll = oracle.synth_middle_stream(n_long, pmtu=4096)
    bs, _, ls = oracle.synth_middle_stream(n_short, pmtu=256, payload_key=0xBEEF)
    buf = np.concatenate([bl, bs])
    lens = np.concatenate([ll, ls]).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    assert int(off[-1]) + int(lens[-1]) == buf.size
    want = oracle_icrcs(buf, off, lens)
    engine.set_variant(variant)
    try:
        out, nerr, after = run_batch(engine, buf, off, lens, write_trailer=True)
        assert nerr == 0
        assert np.array_equal(out, want)
        tr = np.stack([after[int(o) + int(L) - 4: int(o) + int(L)] for o, L in zip(off, lens)])
        assert np.array_equal(tr.view("<u4").ravel(), want)
        flips = [5, n_long + 7]
        for i in flips:
            after[int(off[i]) + 100] ^= 0x10
        d_buf, d_off, d_len = dev(after), dev(off), dev(lens)
        d_ok = torch.zeros(len(lens), dtype=torch.uint8, device="cuda")
        engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(lens), d_ok.data_ptr(),
                            zero_trailer=True, stream=stream_handle())
        torch.cuda.synchronize()
        ok = d_ok.cpu().numpy()
        expect = np.ones(len(lens), np.uint8)
        expect[flips] = 0
        assert np.array_equal(ok, expect)
        zb = d_buf.cpu().numpy()
        assert all(not zb[int(o) + int(L) - 4: int(o) + int(L)].any() for o, L in zip(off, lens))
    finally:
        engine.set_variant(-1)


def _residue_boundary_lengths():
    """Packet lengths (4-byte multiples) where the verify stream (1 + L / 4 words: the trailer is
    its last word, kIcrcResidue) crosses a row boundary of the oct kernel (8-word rows, 10-row
    frames, L <= 1088) or of the one-packet pipeline (64-word rows, 17 rows: L <= 4348 on the fast
    path, 4352 and up on the byte-wise one)."""
    ls = set(range(44, 1201, 4))
    for k in range(1, 19):
        for nv in (64 * k - 1, 64 * k, 64 * k + 1):
            L = 4 * (nv - 1)
            if L >= 44:
                ls.add(L)
    ls.update(range(4336, 4372, 4))
    return np.array(sorted(ls), np.uint32)


@pytest.mark.parametrize("variant", [-1, 16, 40])
@pytest.mark.parametrize("zero_trailer", [False, True])
def test_verify_residue_row_boundaries(engine, variant, zero_trailer):
    """Verify runs as a compute over the packet and its trailer (ICRC residue 0x2144DF1C): every
    row-boundary length of both kernels, right trailers, a flipped payload bit, a flipped trailer
    bit, ragged (default hybrid dispatch or a forced kernel) and strided per length."""
    rng = np.random.default_rng(7 + variant + (1000 if zero_trailer else 0))
    lens = np.repeat(_residue_boundary_lengths(), 2)
    n = lens.size
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
    tr = (off + lens.astype(np.uint64) - 4).astype(np.int64)[:, None] + np.arange(4)
    buf[tr] = oracle_icrcs(buf, off, lens).view(np.uint8).reshape(-1, 4)
    bad_payload = rng.choice(n, 40, replace=False)
    bad_trailer = np.setdiff1d(rng.choice(n, 40, replace=False), bad_payload)
    for i in bad_payload:
        buf[int(off[i]) + 40 + int(rng.integers(0, int(lens[i]) - 44))] ^= 0x10
    for i in bad_trailer:
        buf[int(off[i] + lens[i]) - 4 + int(rng.integers(0, 4))] ^= 0x01
    want = np.ones(n, np.uint8)
    want[bad_payload] = 0
    want[bad_trailer] = 0
    engine.set_variant(variant)
    try:
        d_b, d_o, d_l = dev(buf), dev(off), dev(lens)
        d_ok = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        engine.verify_batch(d_b.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), n, d_ok.data_ptr(), zero_trailer=zero_trailer,
                            stream=stream_handle())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_ok.cpu().numpy(), want)
        if zero_trailer:
            assert not d_b.cpu().numpy()[tr].any()
        # strided, one batch per length (the strided dispatch: oct below 1089 B, one packet per wave above)
        for L in (44, 316, 1084, 1088, 1092, 4152, 4156, 4348, 4352):
            m = 96
            sb = rng.integers(0, 256, m * L, dtype=np.uint8)
            so = np.arange(m, dtype=np.uint64) * L
            sl = np.full(m, L, np.uint32)
            str_ = (so + L - 4).astype(np.int64)[:, None] + np.arange(4)
            sb[str_] = oracle_icrcs(sb, so, sl).view(np.uint8).reshape(-1, 4)
            sb[L * 5 + 40 + (L - 44) // 2] ^= 0x80  # a payload byte of packet 5
            sb[L * 9 + L - 2] ^= 0x04
            d = dev(sb)
            ok = torch.zeros(m, dtype=torch.uint8, device="cuda")
            engine.verify_strided(d.data_ptr(), L, L, m, ok.data_ptr(), zero_trailer=zero_trailer, stream=stream_handle())
            torch.cuda.synchronize()
            w = np.ones(m, np.uint8)
            w[[5, 9]] = 0
            np.testing.assert_array_equal(ok.cpu().numpy(), w, err_msg=f"strided L={L}")
    finally:
        engine.set_variant(-1)


def test_large_mixed_mtu_batch_oct_result_flushes(engine):
    """A C2-shaped batch big enough that every oct wave walks more than kOctRes (8) blocks, so its
    register-buffered block results are stored from inside the ring as well as after it: the
    default hybrid launch against the one-packet pipeline (forced variant 16) on every packet and
    against the oracle on a sample; then trailers written by the default dispatch verify clean,
    and flipped bits are caught exactly."""
    import icrc_amd

    n = 3 << 20  # 768 packets per oct wave: 12 blocks
    w = icrc_amd.workloads.mixed_mtu_stream(n, seed=99)
    s = stream_handle()
    d_buf = icrc_amd.workloads.synthesize(engine, w, stream=s)
    d_off, d_len = dev(w.off), dev(w.lens)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    ref = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, out.data_ptr(), stream=s)
    engine.set_variant(16)
    try:
        engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, ref.data_ptr(), stream=s)
    finally:
        engine.set_variant(-1)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    rng = np.random.default_rng(3)
    pick = np.unique(np.concatenate([np.arange(2048), np.arange(n - 2048, n), rng.choice(n, 20000, replace=False)]))
    lo = w.off[pick].astype(np.int64)
    span = w.lens[pick].astype(np.int64)
    idx = np.concatenate([np.arange(a, a + b) for a, b in zip(lo, span)])
    host = d_buf[torch.from_numpy(idx).cuda()].cpu().numpy()
    soff = np.zeros(pick.size, np.uint64)
    soff[1:] = np.cumsum(span[:-1]).astype(np.uint64)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32)[pick], oracle_icrcs(host, soff, w.lens[pick]))
    # trailers by the default dispatch, then verify through it: clean, then with flipped bits
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, out.data_ptr(), write_trailer=True,
                         stream=s)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, ok.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert bool((ok == 1).all())
    bad = rng.choice(n, 500, replace=False)
    pos = (w.off[bad] + 40 + (w.lens[bad] - 44) // 2).astype(np.int64)
    d_buf[torch.from_numpy(pos).cuda()] ^= 0x20
    engine.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, ok.data_ptr(), stream=s)
    torch.cuda.synchronize()
    want = np.ones(n, np.uint8)
    want[bad] = 0
    np.testing.assert_array_equal(ok.cpu().numpy(), want)
