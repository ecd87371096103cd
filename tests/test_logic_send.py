"""rust_driver's send rule (BlueRDMALogic::send, rust_driver/src/device/software/logic.rs:109-277)
pinned to the reference's own test, test_logic.rs:44-359 (tests/golden/logic_send_cases.json), on
the CPU: the oracle's restatement, its packets decoded by the oracle's receive parse, and the
packetizer kernel's header formulas (kernel_emu) against the oracle's packet bytes.  The GPU
packetizer runs the same cases in test_gpu_logic_send.py."""
import numpy as np
import pytest

import kernel_emu
import logic_cases
import oracle

CASES = logic_cases.load()


def test_fixture_is_the_reference_test():
    assert [c["name"] for c in CASES] == [
        "write_only", "write_first_last_va512", "write_va1023_len4096", "read_response_va1023_len4096",
        "write_only_with_imm", "read_request", "large_64k_two_descriptors", "first_short_total_33k"]
    assert [c["count"] for c in CASES] == [1, 2, 5, 5, 1, 1, 16, 9]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_logic_send_meets_reference_asserts(case):
    msgs = []
    for d in case["descs"]:
        sg = sum(int(s[1]) for s in d["sges"])
        if d["opcode"] == "Read":  # send_read_packet (logic.rs:136-164)
            a, ln, key = d["sges"][0]
            msgs.append(dict(opcode=0x0C, psn=d["psn"], reth_va=d["raddr"], reth_len=d["total_len"],
                             reth_rkey=d["rkey"], imm=None, sec_va=a, sec_len=ln, sec_rkey=key, payload_len=0,
                             payload_start=0))
            continue
        for p in oracle.logic_send(raddr=d["raddr"], total_len=d["total_len"], sge_len=sg, pmtu=d["pmtu"],
                                   psn=d["psn"], is_resp=d["opcode"] == "ReadResp", is_first=d["is_first"],
                                   is_last=d["is_last"], imm=d.get("imm")):
            msgs.append(dict(p, reth_rkey=d["rkey"], payload_start=p["payload_off"], sec_va=None, sec_len=None,
                             sec_rkey=None))
    logic_cases.check(case, msgs)


def _oracle_wire(case):
    import icrc_amd

    specs, nsrc = logic_cases.write_specs(case)
    msgs = icrc_amd.write_messages(specs)
    rng = np.random.default_rng(len(case["name"]))
    src = rng.integers(0, 256, nsrc, dtype=np.uint8)
    wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1])
    wire, lens, icrcs = oracle.send_messages(src, msgs, wire_bytes)
    return msgs, src, wire, lens, icrcs


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_packets_decode_to_reference_asserts(case):
    """The oracle's packets (PacketWriter restatement) decoded by its receive parse
    (to_rdma_message) meet the reference's assertions; ICRCs verify."""
    msgs, src, wire, lens, icrcs = _oracle_wire(case)
    off = logic_cases.packet_offsets(msgs)
    desc = oracle.rx_parse(wire.copy(), off, lens)
    assert np.all(desc["icrc_ok"] == 1) and np.all(desc["status"] == 0)
    starts = []
    k = 0
    for m, d in zip(msgs, case["descs"]):
        for s in range(int(m["npackets"])):
            st = (int(desc[k]["reth_va"]) - int(d["raddr"])) if int(m["kind"]) != 2 else 0
            po = int(desc[k]["payload_offset"])
            pl = int(desc[k]["payload_len"])
            np.testing.assert_array_equal(wire[po: po + pl], src[int(m["payload_offset"]) + st: int(m["payload_offset"]) + st + pl])
            starts.append(st)
            k += 1
    logic_cases.check(case, logic_cases.messages_from_rx(desc, starts))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_kernel_header_formulas_match_oracle(case):
    msgs, src, wire, lens, icrcs = _oracle_wire(case)
    for m in msgs:
        for s in range(int(m["npackets"])):
            words, ln, L = kernel_emu.packetizer_header_words(m, s)
            k = int(m["first_packet"]) + s
            assert L == lens[k]
            o = int(m["out_offset"]) + s * int(m["slot_stride"])
            hdr = np.array(words, dtype="<u4").view(np.uint8)
            np.testing.assert_array_equal(hdr, wire[o: o + hdr.size])


def test_emulator_rule_unchanged_without_flag():
    """Without ICRC_WRITE_RUST_DRIVER the descriptor flags are ignored: the emulator's Write::handle
    rule (ack_req on LAST, RETH len = common.total_len on every packet, common.rs:113)."""
    import icrc_amd

    case = CASES[6]
    specs, nsrc = logic_cases.write_specs(case, rust_driver_flag=0)
    msgs = icrc_amd.write_messages(specs)
    for m in msgs:
        n = int(m["npackets"])
        for s in range(n):
            words, ln, L = kernel_emu.packetizer_header_words(m, s)
            op = words[7] & 0x1F
            assert op == (0x06 if s == 0 else 0x08 if s == n - 1 else 0x07)
            assert kernel_emu._bswap32(words[13]) == int(m["reth_len"])


# ---- test_packet.rs serialisation direction through the product's icrc_packet_headers (host code) ----
def test_pkt_processor_to_buf():
    """rust_driver/src/device/software/tests/test_packet.rs:225-267: set_from_rdma_message of a
    WRITE_FIRST message (dqpn 3, psn 0x123456, pkey 0, RETH 0x1234567812345678 / 0x12345678 /
    0x12345678, 512-byte payload) writes BTH + RETH (28 bytes) that read back as those fields."""
    import icrc_amd

    data = np.ones(512, np.uint8)
    m = icrc_amd.RdmaMsg()
    m.kind, m.opcode, m.tran_type, m.solicited, m.ack_req = 0, 0x06, 0, 0, 0
    m.pkey, m.dqpn, m.psn = 0, 3, 0x123456
    m.reth_va, m.reth_rkey, m.reth_len = 0x1234567812345678, 0x12345678, 0x12345678
    m.payload, m.payload_len = data.ctypes.data, data.size
    hdr, L = icrc_amd.packet_headers(m, "192.168.0.2", 4791, "192.168.0.3", 4791, 1)
    bth = hdr[28:]
    assert bth.size == 12 + 16                                   # size == BTH_SIZE + RETH_SIZE (:254)
    assert bth[0] & 0x1F == 0x06                                 # get_opcode (:257)
    assert int.from_bytes(bytes(bth[4:8]), "big") & 0xFFFFFF == 3  # get_destination_qpn (:258)
    assert int.from_bytes(bytes(bth[8:12]), "big") & 0xFFFFFF == 0x123456  # get_psn (:259)
    assert not bth[8] & 0x80                                     # get_ack_req (:260)
    assert int.from_bytes(bytes(bth[2:4]), "big") == 0           # get_pkey (:261)
    assert int.from_bytes(bytes(bth[12:20]), "big") == 0x1234567812345678  # get_va (:264)
    assert int.from_bytes(bytes(bth[20:24]), "big") == 0x12345678          # get_rkey (:265)
    assert int.from_bytes(bytes(bth[24:28]), "big") == 0x12345678          # get_dlen (:266)
    assert L == 28 + 28 + 512 + 4


def test_set_from_rdma_message_round_trips():
    """test_packet.rs:52-55, :99-102, :148-151, :186-189 — parse (oracle's to_rdma_message) then
    serialise (the product's icrc_packet_headers): the header bytes come back unchanged."""
    import icrc_amd
    import rx_cases

    for name, pkt, _ in rx_cases.reference_cases():
        d = oracle.rx_parse(pkt.copy(), [0], [pkt.size])[0]
        assert d["status"] == 0 and d["icrc_ok"] == 1, name
        hdr, L = icrc_amd.packet_headers(logic_cases.rdma_msg_from_desc(icrc_amd, d), "192.168.0.2", 4791, "192.168.0.3",
                                         4791, 1)
        assert L == pkt.size, name
        np.testing.assert_array_equal(hdr, pkt[: hdr.size], err_msg=name)
