"""Generate tests/golden/logic_send_cases.json — the send-side segmentation cases the REFERENCE's
own test pins: rust_driver/src/device/software/tests/test_logic.rs:44-359 (`test_logic_send`).

Each case is the descriptor(s) the test builds with ToCardWorkRbDescBuilder (tests/mod.rs:52-210;
defaults: qp_type RC, is_first = is_last = true, msn 0, dqp_ip 127.0.0.1) and the fields its
`assert_eq!`s check on the RdmaMessages BlueRDMALogic::send hands to the fake NetSendAgent
(DummpyProxy, test_logic.rs:15-42), in order.  Both are copied as data, with the test_logic.rs line
of each case; nothing here is computed.  A field a case does not assert is absent.

  count           number of messages sent (agent.message.borrow().len())
  opcode          meta_data.get_opcode() (ToHostWorkRbDescOpcode, rust_driver/src/device/types.rs)
  payload_len     message.payload.get_length()
  psn             common_meta().psn
  reth_va / reth_len / reth_rkey, imm, sec_va / sec_len / sec_rkey     General metadata
  psn_consecutive psn of message i+1 == psn of message i + 1 (test_logic.rs:167-191)
  sge0_addr       payload.get_sg_list()[0].data: the payload starts at the first SGE

test_logic_send_raw (test_logic.rs:361-395) is a raw-packet pass-through (send_raw, no RDMA
headers, no ICRC) and is not a packetizer case.

Run from the repo root:  python tests/golden/make_logic_cases.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

WRITE_FIRST, WRITE_MIDDLE, WRITE_LAST, WRITE_ONLY, WRITE_ONLY_IMM = 0x06, 0x07, 0x08, 0x0A, 0x0B
READ_REQUEST, RR_FIRST, RR_MIDDLE, RR_LAST = 0x0C, 0x0D, 0x0E, 0x0F
MTU1024, MTU4096 = 1024, 4096


def desc(opcode, total_len, raddr, pmtu, psn, sges, rkey=1234, dqpn=12, is_first=True, is_last=True, imm=None):
    d = dict(opcode=opcode, total_len=total_len, raddr=raddr, rkey=rkey, pmtu=pmtu, psn=psn, dqpn=dqpn,
             sges=[list(s) for s in sges], is_first=is_first, is_last=is_last)
    if imm is not None:
        d["imm"] = imm
    return d


def cases():
    out = []
    out.append(dict(
        name="write_only", ref="test_logic.rs:51-70",
        descs=[desc("Write", 512, 0, MTU1024, 1234, [(0x1000, 512, 0x1234)])],
        count=1, expect=[dict(opcode=WRITE_ONLY, payload_len=512, sge0_addr=0x1000)]))
    out.append(dict(
        name="write_first_last_va512", ref="test_logic.rs:72-97",
        descs=[desc("Write", 1024, 512, MTU1024, 1234, [(0x1000, 256, 0x1234), (0x2000, 768, 0x1234)])],
        count=2, expect=[dict(opcode=WRITE_FIRST, payload_len=512), dict(opcode=WRITE_LAST, payload_len=512)]))
    out.append(dict(
        name="write_va1023_len4096", ref="test_logic.rs:99-144",
        descs=[desc("Write", 4096, 1023, MTU1024, 1234, [(0x1000, 4096, 0x1234)])],
        count=5, expect=[dict(opcode=WRITE_FIRST, payload_len=1)] + [dict(opcode=WRITE_MIDDLE, payload_len=1024)] * 3
        + [dict(opcode=WRITE_LAST, payload_len=1023)]))
    out.append(dict(
        name="read_response_va1023_len4096", ref="test_logic.rs:146-198",
        descs=[desc("ReadResp", 4096, 1023, MTU1024, 1234, [(0x1000, 4096, 0x1234)])],
        count=5, psn_consecutive=True,
        expect=[dict(opcode=RR_FIRST, payload_len=1)] + [dict(opcode=RR_MIDDLE, payload_len=1024)] * 3
        + [dict(opcode=RR_LAST, payload_len=1023)]))
    out.append(dict(
        name="write_only_with_imm", ref="test_logic.rs:200-226",
        descs=[desc("WriteWithImm", 20, 0, MTU1024, 1234, [(0x1000, 20, 0x1234)], imm=0x1234)],
        count=1, expect=[dict(opcode=WRITE_ONLY_IMM, imm=0x1234)]))
    out.append(dict(
        name="read_request", ref="test_logic.rs:228-256",
        descs=[desc("Read", 1024, 0, MTU1024, 1234, [(0x1000, 1024, 4567)])],
        count=1, expect=[dict(opcode=READ_REQUEST, reth_va=0, reth_len=1024, reth_rkey=1234, sec_va=0x1000,
                              sec_len=1024, sec_rkey=4567)]))
    out.append(dict(
        name="large_64k_two_descriptors", ref="test_logic.rs:258-308",
        descs=[desc("Write", 1024 * 64, 0, MTU4096, 0, [(0, 1024 * 32, 0x1234)], is_last=False),
               desc("Write", 1024 * 32, 1024 * 32, MTU4096, 8, [(0, 1024 * 32, 0x1234)], is_first=False)],
        count=16,
        expect=[dict(opcode=WRITE_FIRST, payload_len=4096, psn=0, reth_va=0, reth_len=1024 * 64, reth_rkey=1234)]
        + [dict(opcode=WRITE_MIDDLE, psn=i, payload_len=4096) for i in range(1, 15)]
        + [dict(opcode=WRITE_LAST, psn=15, payload_len=1024 * 4)]))
    out.append(dict(
        name="first_short_total_33k", ref="test_logic.rs:309-358",
        descs=[desc("Write", 1024 * 33, 1024 * 31, MTU4096, 0, [(0, 1024, 0x1234)], is_last=False),
               desc("Write", 1024 * 32, 1024 * 32, MTU4096, 1, [(1024 * 32, 1024 * 32, 0x1234)], is_first=False)],
        count=9,
        expect=[dict(opcode=WRITE_FIRST, psn=0, payload_len=1024, reth_va=1024 * 31, reth_len=1024 * 33,
                     reth_rkey=1234)]
        + [dict(opcode=WRITE_MIDDLE, psn=i, payload_len=4096) for i in range(1, 8)]
        + [dict(opcode=WRITE_LAST, psn=8, payload_len=1024 * 4)]))
    return out


def main():
    path = os.path.join(HERE, "logic_send_cases.json")
    with open(path, "w") as f:
        json.dump(cases(), f, indent=1)
        f.write("\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
