"""The fused send packetizer under ICRC_WRITE_RUST_DRIVER, pinned to the reference's own send test
(rust_driver/src/device/software/tests/test_logic.rs:44-359, tests/golden/logic_send_cases.json),
and the header serialisation pinned to test_packet.rs's set_from_rdma_message round trips
(:52-55, :99-102, :148-151, :186-189) with the packets decoded by the product's receive parse.

Per case: icrc_write_packetize_device emits the packets; every byte equals the oracle's
restatement (BlueRDMALogic::send -> PacketWriter::write); icrc_rx_parse_device decodes them and the
decoded fields meet the reference test's assertions (count, opcode, payload length, PSN, RETH
va/len/rkey, ImmDt, secondary RETH)."""
import numpy as np
import pytest

import logic_cases
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = logic_cases.load()


def dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def stream_handle():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_packetizer_reference_logic_cases(engine, case):
    import icrc_amd

    specs, nsrc = logic_cases.write_specs(case)
    msgs = icrc_amd.write_messages(specs)
    npk = int(msgs["npackets"].sum())
    assert npk == case["count"]
    rng = np.random.default_rng(len(case["name"]) + 100)
    src = rng.integers(0, 256, nsrc, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1])
    d_src, d_msgs = dev(src), dev(msgs.view(np.uint8))
    d_wire = torch.full((wire_bytes,), 0xEE, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
    s = stream_handle()
    engine.packetize(d_src.data_ptr(), src.size, d_msgs.data_ptr(), len(msgs), npk, d_wire.data_ptr(), wire_bytes,
                     d_len.data_ptr(), d_icrc.data_ptr(), stream=s)
    torch.cuda.synchronize()
    lens = d_len.cpu().numpy().view(np.uint32)
    wire = d_wire.cpu().numpy()
    want_wire, want_lens, want_icrc = oracle.send_messages(src, msgs, wire_bytes)
    np.testing.assert_array_equal(lens, want_lens)
    np.testing.assert_array_equal(d_icrc.cpu().numpy().view(np.uint32), want_icrc)
    off = logic_cases.packet_offsets(msgs)
    for k in range(npk):  # every packet byte; nothing written past a packet inside its slot
        o, L = int(off[k]), int(lens[k])
        np.testing.assert_array_equal(wire[o: o + L], want_wire[o: o + L])
        slot_end = o + int(msgs["slot_stride"][np.searchsorted(msgs["first_packet"], k, side="right") - 1])
        assert np.all(wire[o + L: min(slot_end, wire_bytes)] == 0xEE)
    # decode with the product's receive parse; the reference test's assertions on the fields
    d_off = dev(off)
    d_desc = torch.zeros(npk * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(npk, dtype=torch.uint8, device="cuda")
    engine.rx_parse(d_wire.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), npk, d_desc.data_ptr(), d_ok.data_ptr(),
                    stream=s)
    torch.cuda.synchronize()
    desc = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    assert np.all(d_ok.cpu().numpy() == 1) and np.all(desc["status"] == 0)
    starts, k = [], 0
    for m, d in zip(msgs, case["descs"]):
        for _ in range(int(m["npackets"])):
            st = int(desc[k]["reth_va"]) - int(d["raddr"]) if int(m["kind"]) != 2 else 0
            po, pl = int(desc[k]["payload_offset"]), int(desc[k]["payload_len"])
            base = int(m["payload_offset"]) + st
            np.testing.assert_array_equal(wire[po: po + pl], src[base: base + pl])
            starts.append(st)
            k += 1
    logic_cases.check(case, logic_cases.messages_from_rx(desc, starts))


def test_packetizer_reference_logic_cases_batched(engine):
    """All cases' descriptors in ONE launch (mixed kinds, flags, PMTUs): same bytes as the oracle."""
    import icrc_amd

    specs, srcs, base = [], [], 0
    for c in CASES:
        sp, n = logic_cases.write_specs(c)
        for x in sp:
            if x["kind"] != 2:
                x["payload_offset"] += base
        specs += sp
        base += n
    msgs = icrc_amd.write_messages(specs)
    npk = int(msgs["npackets"].sum())
    src = np.random.default_rng(9).integers(0, 256, base, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1])
    d_src, d_msgs = dev(src), dev(msgs.view(np.uint8))
    d_wire = torch.zeros(wire_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    engine.packetize(d_src.data_ptr(), src.size, d_msgs.data_ptr(), len(msgs), npk, d_wire.data_ptr(), wire_bytes,
                     d_len.data_ptr(), 0, stream=stream_handle())
    torch.cuda.synchronize()
    want_wire, want_lens, _ = oracle.send_messages(src, msgs, wire_bytes)
    np.testing.assert_array_equal(d_len.cpu().numpy().view(np.uint32), want_lens)
    np.testing.assert_array_equal(d_wire.cpu().numpy(), want_wire)


@pytest.mark.parametrize("seed", [0, 1])
def test_packetizer_rust_driver_random_vs_oracle(engine, seed):
    """Random rust_driver descriptors (any raddr alignment, PMTU 256..4096, lengths 0..70000, is_first /
    is_last / imm, WRITE and READ RESPONSE, IPv4 checksum fill, UDP-payload-only form): every byte of
    every packet against the oracle's BlueRDMALogic::send restatement."""
    import icrc_amd

    rng = np.random.default_rng(1000 + seed)
    specs, pos = [], 0
    for i in range(300):
        total = int(rng.choice([0, 1, 3, 4, 255, 256, 257, 1023, 4096, 4097, int(rng.integers(0, 70000))]))
        kind = int(rng.integers(0, 2))
        flags = 0x02 | int(rng.choice([0, 0x20, 0x40, 0x60])) | (0x80 if kind == 0 and rng.random() < 0.4 else 0)
        flags |= int(rng.choice([0, 0x01, 0x04, 0x08, 0x10]))
        specs.append(dict(local_va=int(rng.integers(0, 1 << 48)), remote_va=int(rng.integers(0, 1 << 64, dtype=np.uint64)),
                          payload_offset=pos, total_len=total, reth_len=int(rng.integers(0, 1 << 32)),
                          pmtu=int(rng.choice([256, 512, 1024, 2048, 4096])), rkey=int(rng.integers(0, 1 << 32)),
                          dqpn=int(rng.integers(0, 1 << 24)), psn=int(rng.integers(0, 1 << 24)),
                          msn=int(rng.integers(0, 1 << 16)), dst_ip=int(rng.integers(0, 1 << 32)), kind=kind,
                          flags=flags, imm=int(rng.integers(0, 1 << 32)), ip_id=int(rng.integers(0, 1 << 16))))
        pos += total + int(rng.integers(0, 3)) * 4
    msgs = icrc_amd.write_messages(specs)
    npk = int(msgs["npackets"].sum())
    src = rng.integers(0, 256, pos + 8, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1])
    d_src, d_msgs = dev(src), dev(msgs.view(np.uint8))
    d_wire = torch.zeros(wire_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
    engine.packetize(d_src.data_ptr(), src.size, d_msgs.data_ptr(), len(msgs), npk, d_wire.data_ptr(), wire_bytes,
                     d_len.data_ptr(), d_icrc.data_ptr(), stream=stream_handle())
    torch.cuda.synchronize()
    want_wire, want_lens, want_icrc = _oracle_udp_form(src, msgs, wire_bytes)
    np.testing.assert_array_equal(d_len.cpu().numpy().view(np.uint32), want_lens)
    np.testing.assert_array_equal(d_icrc.cpu().numpy().view(np.uint32), want_icrc)
    np.testing.assert_array_equal(d_wire.cpu().numpy(), want_wire)


def _oracle_udp_form(src, msgs, wire_bytes):
    """oracle.send_messages, with messages flagged ICRC_WRITE_UDP_PAYLOAD_ONLY moved to the form the
    packetizer stores for them (packet bytes [28, L) at the slot; length L - 28)."""
    full = msgs.copy()
    full["flags"] &= ~np.uint8(0x10)
    wire, lens, icrcs = oracle.send_messages(src, full, wire_bytes + 64)
    out = np.zeros(wire_bytes, np.uint8)
    lens = lens.copy()
    for m in msgs:
        for s in range(int(m["npackets"])):
            k = int(m["first_packet"]) + s
            o = int(m["out_offset"]) + s * int(m["slot_stride"])
            L = int(lens[k])
            if L == 0:
                continue
            if int(m["flags"]) & 0x10:
                out[o: o + L - 28] = wire[o + 28: o + L]
                lens[k] = L - 28
            else:
                out[o: o + L] = wire[o: o + L]
    return out, lens, icrcs


# ---- test_packet.rs: set_from_rdma_message round trips and test_pkt_processor_to_buf ------------
def test_set_from_rdma_message_round_trips_on_device(engine):
    """test_packet.rs:52-55, :99-102, :148-151, :186-189: a buffer the setters filled, parsed by
    to_rdma_message (here icrc_rx_parse_device on the GPU) and written back by set_from_rdma_message
    (here icrc_packet_headers), gives the same header bytes."""
    import icrc_amd
    import rx_cases

    cases = rx_cases.reference_cases()
    pkts = [p for _, p, _ in cases]
    lens = np.array([p.size for p in pkts], np.uint32)
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum((lens[:-1].astype(np.uint64) + 3) // 4 * 4)
    buf = np.zeros(int(off[-1]) + int(lens[-1]) + 8, np.uint8)
    for o, p in zip(off, pkts):
        buf[int(o): int(o) + p.size] = p
    d_buf, d_off, d_len = dev(buf), dev(off), dev(lens)
    d_desc = torch.zeros(lens.size * 72, dtype=torch.uint8, device="cuda")
    engine.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), lens.size, d_desc.data_ptr(),
                    stream=stream_handle())
    torch.cuda.synchronize()
    desc = d_desc.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    for (name, pkt, _), d in zip(cases, desc):
        m = logic_cases.rdma_msg_from_desc(icrc_amd, d)
        hdr, L = icrc_amd.packet_headers(m, "192.168.0.2", 4791, "192.168.0.3", 4791, 1)
        assert L == pkt.size, name
        size = hdr.size - 28  # size_of the composite header (BTH_SIZE + ...)
        assert size == {0x06: 28, 0x09: 32, 0x0C: 44, 0x11: 16}[int(d["opcode"])], name
        np.testing.assert_array_equal(hdr[28:], pkt[28: 28 + size], err_msg=name)
