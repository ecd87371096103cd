"""logic_cases.py — the reference's send-segmentation cases (rust_driver/src/device/software/tests/
test_logic.rs:44-359, committed as data in tests/golden/logic_send_cases.json by
tests/golden/make_logic_cases.py) as packetizer inputs, and the check of sent messages against the
reference's own assertions."""
import json
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "logic_send_cases.json")
LOCALHOST = 0x7F000001  # ToCardWorkRbDescBuilder: dqp_ip = Ipv4Addr::LOCALHOST (tests/mod.rs:160)
SRC_IP = 0xC0A80002


def load():
    with open(_PATH) as f:
        return json.load(f)


def write_specs(case, rust_driver_flag=0x02):
    """icrc_write_msg specs (include/icrc.h) for a case's descriptors, their SG lists laid out back
    to back in one source buffer.  Returns (specs, src_bytes)."""
    specs, pos = [], 0
    for d in case["descs"]:
        sg_total = sum(int(s[1]) for s in d["sges"])
        flags = rust_driver_flag
        if not d["is_first"]:
            flags |= 0x20
        if not d["is_last"]:
            flags |= 0x40
        spec = dict(remote_va=int(d["raddr"]), rkey=int(d["rkey"]), pmtu=int(d["pmtu"]), psn=int(d["psn"]),
                    dqpn=int(d["dqpn"]), msn=0, dst_ip=LOCALHOST, src_ip=SRC_IP, ip_id=1, reth_len=int(d["total_len"]))
        if d["opcode"] == "Read":  # send_read_packet (logic.rs:136-164): RETH + secondary RETH (the local SGE)
            a, ln, key = d["sges"][0]
            spec.update(kind=2, local_va=int(a), lkey=int(key), total_len=int(ln), payload_offset=0)
        else:
            spec.update(kind=1 if d["opcode"] == "ReadResp" else 0, local_va=int(d["sges"][0][0]),
                        total_len=sg_total, payload_offset=pos)
            if d["opcode"] == "WriteWithImm":
                flags |= 0x80
                spec["imm"] = int(d["imm"])
            pos += sg_total
        spec["flags"] = flags
        specs.append(spec)
    return specs, max(pos, 4)


def check(case, msgs):
    """msgs: the sent messages in order, dicts with opcode, payload_len, psn, reth_va, reth_len,
    reth_rkey, imm (None when absent), sec_va/sec_len/sec_rkey, payload_start (offset of the
    payload's first byte in the descriptor's SG list)."""
    name = case["name"] + " (" + case["ref"] + ")"
    assert len(msgs) == case["count"], (name, len(msgs))
    for i, (got, want) in enumerate(zip(msgs, case["expect"])):
        for k, v in want.items():
            if k == "sge0_addr":  # payload.get_sg_list()[0].data: the payload starts at the first SGE
                assert got["payload_start"] == 0, (name, i, k)
            else:
                assert got[k] is not None and int(got[k]) == int(v), (name, i, k, got[k], v)
    if case.get("psn_consecutive"):
        for a, b in zip(msgs, msgs[1:]):
            assert int(b["psn"]) == (int(a["psn"]) + 1) & 0xFFFFFF, name


def messages_from_rx(desc, payload_starts):
    """RX_DESC_DTYPE records (the receive parse of the sent packets) -> check() dicts."""
    out = []
    for d, ps in zip(desc, payload_starts):
        fl = int(d["flags"])
        out.append(dict(opcode=int(d["opcode"]), payload_len=int(d["payload_len"]), psn=int(d["psn"]),
                        reth_va=int(d["reth_va"]), reth_len=int(d["reth_len"]), reth_rkey=int(d["reth_rkey"]),
                        imm=int(d["imm"]) if fl & 0x04 else None,
                        sec_va=int(d["sec_va"]) if fl & 0x08 else None,
                        sec_len=int(d["sec_len"]) if fl & 0x08 else None,
                        sec_rkey=int(d["sec_rkey"]) if fl & 0x08 else None, payload_start=ps))
    return out


def packet_offsets(msgs):
    return np.concatenate([int(m["out_offset"]) + np.arange(int(m["npackets"]), dtype=np.uint64) * int(m["slot_stride"])
                           for m in msgs]).astype(np.uint64)


def rdma_msg_from_desc(icrc_amd, d):
    """RdmaMessage from a parsed descriptor (the metadata to_rdma_message returns)."""
    m = icrc_amd.RdmaMsg()
    fl = int(d["flags"])
    m.kind = 1 if fl & 0x10 else 0
    m.opcode = int(d["opcode"])
    m.tran_type = int(d["tran_type"])
    m.solicited = 1 if fl & 0x01 else 0
    m.ack_req = 1 if fl & 0x02 else 0
    m.pkey = int(d["pkey"])
    m.dqpn = int(d["dqpn"])
    m.psn = int(d["psn"])
    m.aeth_code, m.aeth_value, m.msn = int(d["aeth_code"]), int(d["aeth_value"]), int(d["aeth_msn"])
    m.reth_va, m.reth_rkey, m.reth_len = int(d["reth_va"]), int(d["reth_rkey"]), int(d["reth_len"])
    m.has_imm, m.imm = (1 if fl & 0x04 else 0), int(d["imm"])
    m.has_secondary_reth = 1 if fl & 0x08 else 0
    m.sec_va, m.sec_rkey, m.sec_len = int(d["sec_va"]), int(d["sec_rkey"]), int(d["sec_len"])
    m.payload = None
    m.payload_len = int(d["payload_len"])
    return m
