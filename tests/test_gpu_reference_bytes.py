"""The product's packet writers pinned to bytes the REFERENCE holds (not to the oracle, which is a
second restatement of the same reading):

  KAT1  blue-rdma-device/src/third_party/net/packet_processor.rs:367-378 — a complete 188-byte
        WRITE_ONLY packet (192.168.0.2 -> .3, dqpn 2, solicited, ack_req, va 0x7f7e91000000,
        rkey 0x01709a33, len 128, 128 x 0xFF) with its IPv4 checksum 0xF8DA filled
        (rust_driver/src/responser.rs:388-393 computes that checksum for these header bytes)
  KAT3  blue-rdma-device/src/net/util.rs:227-230 — generate_ack's 20-byte UDP payload, ICRC
        ba 11 c7 23; the 48-byte packet around it from generate_ack's own fields (util.rs:134-170)

and configs[3] at full size: a 16 MiB RDMA WRITE (4096 x 4156-B packets) through compute with
write_trailer then verify with zero_trailer, one flipped bit per 1,024 packets.
"""
import numpy as np
import pytest

import oracle
from golden_kats import KAT1, KAT1_ICRC, KAT3, KAT3_ICRC, KAT3_UDP_PAYLOAD

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def stream_handle():
    return torch.cuda.current_stream().cuda_stream


def kat1_message(icrc_amd, payload: np.ndarray):
    m = icrc_amd.RdmaMsg()
    m.kind = 0
    m.opcode = 0x0A          # RdmaWriteOnly
    m.tran_type = 0          # RC
    m.solicited = 1
    m.ack_req = 1
    m.pkey = 0
    m.dqpn = 2
    m.psn = 0
    m.reth_va = 0x7F7E91000000
    m.reth_rkey = 0x01709A33
    m.reth_len = 128
    m.payload = payload.ctypes.data
    m.payload_len = payload.size
    return m


def test_packet_writer_reproduces_kat1_bytes(engine):
    """PacketWriter::write (icrc_packet_write, ICRC on the GPU) + the batched IPv4 checksum
    (fill) reproduce the reference's KAT1 packet byte for byte."""
    import icrc_amd

    payload = np.full(128, 0xFF, np.uint8)
    buf = np.zeros(8192, np.uint8)
    L = (icrc_amd.PacketWriter(buf).src_addr("192.168.0.2").src_port(4791).dest_addr("192.168.0.3")
         .dest_port(4791).ip_id(1).message(kat1_message(icrc_amd, payload)).write())
    assert L == len(KAT1) == 188
    pkt = buf[:L].copy()
    assert int(pkt[-4:].view("<u4")[0]) == KAT1_ICRC
    want = np.frombuffer(KAT1, np.uint8)
    # PacketWriter leaves the IPv4 checksum 0 (write_ip_udp_header, packet_processor.rs:307-332)
    diff = np.nonzero(pkt != want)[0].tolist()
    assert diff == [10, 11] and pkt[10] == 0 and pkt[11] == 0
    d = dev(pkt)
    d_csum = torch.zeros(1, dtype=torch.int16, device="cuda")
    engine.ipv4_checksum(d.data_ptr(), 1, stride=L, d_csum=d_csum.data_ptr(), fill=True, stream=stream_handle())
    torch.cuda.synchronize()
    assert int(d_csum.cpu().numpy().view(np.uint16)[0]) == 0xF8DA
    np.testing.assert_array_equal(d.cpu().numpy(), want)


def test_packetizer_reproduces_kat1_bytes(engine):
    """The fused send packetizer, given KAT1's message as a one-segment WRITE with the IPv4
    checksum fill and the solicited flag, emits KAT1 byte for byte (trailer included)."""
    import icrc_amd

    src = np.full(128, 0xFF, np.uint8)
    msgs = icrc_amd.write_messages([dict(
        local_va=0x7F7E90000000, remote_va=0x7F7E91000000, payload_offset=0, total_len=128, pmtu=4096,
        rkey=0x01709A33, dqpn=2, psn=0, msn=0, dst_ip=0xC0A80003, kind=0, ip_id=1,
        flags=icrc_amd.WRITE_FILL_IPV4_CSUM | icrc_amd.WRITE_SOLICITED)], slot_stride=192)
    assert int(msgs["npackets"][0]) == 1
    d_src, d_msgs = dev(src), dev(msgs.view(np.uint8))
    d_wire = torch.full((192,), 0xEE, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(1, dtype=torch.int32, device="cuda")
    engine.packetize(d_src.data_ptr(), src.size, d_msgs.data_ptr(), 1, 1, d_wire.data_ptr(), 192,
                     d_len.data_ptr(), d_icrc.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    assert int(d_len.item()) == 188
    assert int(d_icrc.cpu().numpy().view(np.uint32)[0]) == KAT1_ICRC
    wire = d_wire.cpu().numpy()
    np.testing.assert_array_equal(wire[:188], np.frombuffer(KAT1, np.uint8))
    assert np.all(wire[188:] == 0xEE)  # nothing past the packet


def test_packet_writer_reproduces_kat3_ack(engine):
    """generate_ack (net/util.rs:134-170) through icrc_packet_write: the 48-byte packet, and its
    UDP payload equals the reference's captured bytes (util.rs:227-230)."""
    import icrc_amd

    m = icrc_amd.RdmaMsg()
    m.kind = 1               # Metadata::Acknowledge
    m.opcode = 0x11
    m.tran_type = 0
    m.pkey = 0               # msg.meta_data.common_meta().pkey
    m.dqpn = 2               # peer_qpn
    m.psn = 0                # expected_psn
    m.aeth_code = 0          # Ack
    m.aeth_value = 0x1F
    m.msn = 0                # = pkey
    buf = np.zeros(48, np.uint8)
    L = (icrc_amd.PacketWriter(buf).src_addr("192.168.0.3").src_port(4791).dest_addr("192.168.0.2")
         .dest_port(4791).ip_id(1).message(m).write())
    assert L == 48
    np.testing.assert_array_equal(buf, np.frombuffer(KAT3, np.uint8))
    np.testing.assert_array_equal(buf[28:], np.frombuffer(KAT3_UDP_PAYLOAD, np.uint8))
    assert int(buf[-4:].view("<u4")[0]) == KAT3_ICRC


def test_c3_full_size_roundtrip_with_negatives(engine):
    """configs[3] as stated: a 16 MiB WRITE segmented at 4 KiB (4096 packets —
    exactly the small-batch dispatch threshold, num_cu x 16), compute with write_trailer (send),
    verify with zero_trailer (receive), one flipped bit per 1,024 packets; trailers and verdicts
    against the oracle."""
    import icrc_amd

    w = icrc_amd.workloads.write_message(16 << 20, 4096)
    assert w.n == 4096
    s = stream_handle()
    d_buf = icrc_amd.workloads.synthesize(engine, w, stream=s)
    d_off, d_len = dev(w.off), dev(w.lens)
    d_out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
    engine.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_out.data_ptr(),
                         write_trailer=True, stream=s)
    torch.cuda.synchronize()
    host = d_buf.cpu().numpy()
    ref_buf, ref_off, ref_lens = oracle.synth_write(
        16 << 20, 4096, local_va=0x7F7E8EE00000, remote_va=0x7F7E8FC00000, rkey=0x2000003, dqpn=2,
        psn0=0, msn=0, dst_ip=0xC0A80003, payload_key=0xABCDEF)
    np.testing.assert_array_equal(ref_lens, w.lens)
    np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32),
                                  oracle.compute_icrc_batch(ref_buf, ref_off, ref_lens))
    for i in (0, 1, 2047, 4094, 4095):  # whole packets (trailers included) equal the oracle's
        a, b = int(w.off[i]), int(ref_off[i])
        np.testing.assert_array_equal(host[a: a + int(w.lens[i])], ref_buf[b: b + int(ref_lens[i])])
    rng = np.random.default_rng(1024)
    flips = np.arange(0, w.n, 1024) + rng.integers(0, 1024, w.n // 1024)
    for i in flips:  # one flipped payload bit per 1,024 packets
        pos = int(w.off[i]) + 56 + int(rng.integers(0, 4096))
        host[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    d_rx = dev(host)
    d_ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
    engine.verify_batch(d_rx.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_ok.data_ptr(),
                        zero_trailer=True, stream=s)
    torch.cuda.synchronize()
    expect = np.ones(w.n, np.uint8)
    expect[flips] = 0
    np.testing.assert_array_equal(d_ok.cpu().numpy(), expect)
    rx = d_rx.cpu().numpy()
    tr = (w.off + w.lens.astype(np.uint64) - 4).astype(np.int64)[:, None] + np.arange(4)
    assert not rx[tr].any()  # every trailer zeroed (packet_processor.rs:350)
    np.testing.assert_array_equal(np.delete(rx, tr.ravel()), np.delete(host, tr.ravel()))  # nothing else


# ---- receive-side auto-ACK (icrc_ack_from_rx_device) vs generate_ack (net/util.rs:134-170) ----
def _ack_expected(desc, ctx, udp_only=False):
    """The handlers' rule (write_first.rs:35-82): need_ack = can_auto_ack && ack_req, with
    can_auto_ack = QP present && !error && psn == expected_psn; plus status OK / ICRC verified /
    not itself an ACK.  The packet: the oracle's generate_ack restatement."""
    import icrc_amd

    out, lens = {}, np.zeros(desc.size, np.uint32)
    for i, (d, x) in enumerate(zip(desc, ctx)):
        need = (d["status"] == icrc_amd.RX_OK and d["icrc_ok"] == 1 and not d["flags"] & icrc_amd.RX_ACKNOWLEDGE
                and d["flags"] & icrc_amd.RX_ACK_REQ and x["flags"] & 1 and int(d["psn"]) == int(x["expected_psn"]))
        if need:
            pkt, udp = oracle.generate_ack(int(d["pkey"]), int(x["peer_qpn"]), int(x["expected_psn"]))
            out[i] = udp if udp_only else pkt
            lens[i] = out[i].size
    return out, lens


def test_ack_kernel_reproduces_kat3(engine):
    import icrc_amd

    desc = np.zeros(1, icrc_amd.RX_DESC_DTYPE)
    desc["opcode"], desc["flags"], desc["icrc_ok"], desc["status"], desc["pkey"], desc["psn"] = 0x0A, 0x02, 1, 0, 0, 0
    ctx = np.zeros(1, icrc_amd.ACK_CTX_DTYPE)
    ctx["peer_qpn"], ctx["expected_psn"], ctx["flags"] = 2, 0, 1
    for udp_only, want in ((False, KAT3), (True, KAT3_UDP_PAYLOAD)):
        d_out = torch.zeros(64, dtype=torch.uint8, device="cuda")
        d_len = torch.zeros(1, dtype=torch.int32, device="cuda")
        d_desc, d_ctx = dev(desc.view(np.uint8)), dev(ctx.view(np.uint8))  # alive until the kernel has run
        engine.ack_from_rx(d_desc.data_ptr(), d_ctx.data_ptr(), 1, d_out.data_ptr(),
                           64, d_len.data_ptr(), udp_payload_only=udp_only, stream=stream_handle())
        torch.cuda.synchronize()
        assert int(d_len.item()) == len(want)
        np.testing.assert_array_equal(d_out.cpu().numpy()[: len(want)], np.frombuffer(want, np.uint8))


def test_ack_kernel_decision_and_bytes_vs_oracle(engine):
    """Random descriptors (every status, ICRC result, ACK / non-ACK opcodes, ack_req, QP valid or
    not, PSN equal / unequal to the expected one): which packets get an ACK and its bytes."""
    import icrc_amd

    rng = np.random.default_rng(48)
    n = 5000
    desc = np.zeros(n, icrc_amd.RX_DESC_DTYPE)
    desc["status"] = rng.choice([0, 0, 0, 0, 1, 2, 3], n)
    desc["icrc_ok"] = rng.choice([1, 1, 1, 0, 0xFF], n)
    desc["flags"] = rng.integers(0, 32, n)
    desc["pkey"] = rng.integers(0, 1 << 16, n)
    desc["psn"] = rng.integers(0, 1 << 24, n)
    ctx = np.zeros(n, icrc_amd.ACK_CTX_DTYPE)
    ctx["peer_qpn"] = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    ctx["expected_psn"] = np.where(rng.random(n) < 0.7, desc["psn"], rng.integers(0, 1 << 24, n))
    ctx["flags"] = rng.choice([0, 1, 1, 1], n)
    for udp_only, stride in ((False, 48), (True, 20), (False, 64)):
        want, wlen = _ack_expected(desc, ctx, udp_only)
        assert 100 < len(want) < n  # ~4.5 % of the random descriptors qualify
        d_out = torch.full((n * stride,), 0xCD, dtype=torch.uint8, device="cuda")
        d_len = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        d_desc, d_ctx = dev(desc.view(np.uint8)), dev(ctx.view(np.uint8))  # alive until the kernel has run
        engine.ack_from_rx(d_desc.data_ptr(), d_ctx.data_ptr(), n,
                           d_out.data_ptr(), stride, d_len.data_ptr(), udp_payload_only=udp_only,
                           stream=stream_handle())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_len.cpu().numpy().view(np.uint32), wlen)
        out = d_out.cpu().numpy().reshape(n, stride)
        for i in range(n):
            if i in want:
                np.testing.assert_array_equal(out[i, : want[i].size], want[i])
                assert np.all(out[i, want[i].size:] == 0xCD)
            else:
                assert np.all(out[i] == 0xCD)  # no ACK due: slot untouched


def test_receive_then_ack_pipeline(engine):
    """The receive side on the device end to end: the packetizer's WRITE stream (ack_req on each
    message's LAST / ONLY packet) -> icrc_rx_parse_device -> icrc_ack_from_rx_device; one ACK per
    message, for the messages whose QP expects that PSN; a corrupted LAST packet gets none."""
    import icrc_amd

    rng = np.random.default_rng(7)
    specs = [dict(local_va=0x1000 * i, remote_va=0x7F0000000000 + (i << 20), payload_offset=(i * 20000),
                  total_len=int(rng.integers(1, 20000)), pmtu=4096, rkey=9, dqpn=100 + i, psn=int(rng.integers(0, 1 << 24)),
                  msn=i, dst_ip=0xC0A80003, kind=int(rng.integers(0, 2))) for i in range(40)]
    msgs = icrc_amd.write_messages(specs)
    npk = int(msgs["npackets"].sum())
    src = rng.integers(0, 256, 40 * 20000, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1])
    d_src, d_msgs = dev(src), dev(msgs.view(np.uint8))
    d_wire = torch.zeros(wire_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    s = stream_handle()
    engine.packetize(d_src.data_ptr(), src.size, d_msgs.data_ptr(), len(msgs), npk, d_wire.data_ptr(), wire_bytes,
                     d_len.data_ptr(), 0, stream=s)
    torch.cuda.synchronize()
    off = np.concatenate([int(m["out_offset"]) + np.arange(int(m["npackets"]), dtype=np.uint64) * int(m["slot_stride"])
                          for m in msgs]).astype(np.uint64)
    last = (msgs["first_packet"] + msgs["npackets"] - 1).astype(np.int64)
    bad = int(last[3])
    d_wire.view(-1)[int(off[bad]) + 60] ^= 1  # corrupt message 3's LAST packet
    d_desc = torch.zeros(npk * 72, dtype=torch.uint8, device="cuda")
    d_off = dev(off)
    engine.rx_parse(d_wire.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), npk, d_desc.data_ptr(), stream=s)
    # QP state per packet: message i's QP expects its LAST packet's PSN, except every 5th message
    ctx = np.zeros(npk, icrc_amd.ACK_CTX_DTYPE)
    for i, m in enumerate(msgs):
        for k in range(int(m["first_packet"]), int(m["first_packet"] + m["npackets"])):
            ctx[k]["peer_qpn"] = 500 + i
            ctx[k]["flags"] = 1
            lastpsn = (int(m["psn"]) + int(m["npackets"]) - 1) & 0xFFFFFF
            ctx[k]["expected_psn"] = lastpsn if i % 5 else (lastpsn + 1) & 0xFFFFFF
    d_out = torch.zeros(npk * 48, dtype=torch.uint8, device="cuda")
    d_alen = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_ctx = dev(ctx.view(np.uint8))
    engine.ack_from_rx(d_desc.data_ptr(), d_ctx.data_ptr(), npk, d_out.data_ptr(), 48,
                       d_alen.data_ptr(), stream=s)
    torch.cuda.synchronize()
    alen = d_alen.cpu().numpy()
    got_acks = set(np.nonzero(alen)[0].tolist())
    want_acks = {int(last[i]) for i in range(len(msgs)) if i % 5 and int(last[i]) != bad}
    assert got_acks == want_acks
    out = d_out.cpu().numpy().reshape(npk, 48)
    for i, m in enumerate(msgs):
        k = int(last[i])
        if k in want_acks:
            pkt, _ = oracle.generate_ack(int(m["msn"]), 500 + i, int(ctx[k]["expected_psn"]))
            np.testing.assert_array_equal(out[k], pkt)
