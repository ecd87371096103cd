"""rx_cases.py — receive-parse test helpers: a packet corpus over every opcode with corrupted
variants, and a CPU model of the kernel's word-level parse (icrc_kernels.hip rx_store)."""
import numpy as np

import oracle


def emulate(pkt: np.ndarray, off: int) -> np.ndarray:
    """CPU model of rx_store over the header words as the kernel gathers them (zero past L-4)."""
    L = pkt.size
    d = np.zeros(1, dtype=oracle.RX_DESC_DTYPE)[0]
    hb = np.zeros(72, np.uint8)
    n = min(72, max(L - 4, 0))
    hb[:n] = pkt[:n]
    w = hb.view("<u4")
    bs = lambda x: int.from_bytes(int(x).to_bytes(4, "little"), "big")
    status = 3
    if L >= 44:
        w7 = int(w[7]); op, tran, fl = w7 & 0x1F, (w7 >> 5) & 7, (w7 >> 8) & 0xFF
        pad = (fl >> 5) & 3
        hs = 32 if op in (9, 11) else 44 if op == 12 else 16 if op == 17 else 28 if 6 <= op <= 16 else 0
        if hs == 0:
            status = 1
        elif tran > 6:
            status = 2
        elif L - 32 < hs + pad:
            status = 3
        else:
            status = 0
            flags = (1 if fl & 0x80 else 0) | (2 if int(w[9]) & 0x80 else 0)
            d["payload_offset"] = off + 28 + hs
            d["payload_len"] = L - 32 - hs - pad
            d["dqpn"] = bs(w[8]) & 0xFFFFFF
            d["psn"] = bs(w[9]) & 0xFFFFFF
            if hs == 16:
                flags |= 0x10
                d["aeth_code"], d["aeth_value"] = (int(w[10]) >> 5) & 3, int(w[10]) & 0x1F
                d["aeth_msn"] = bs(w[10]) & 0xFFFFFF
            else:
                d["reth_va"] = (bs(w[10]) << 32) | bs(w[11])
                d["reth_rkey"], d["reth_len"] = bs(w[12]), bs(w[13])
                if hs == 32:
                    flags |= 4
                    d["imm"] = bs(w[14])
                elif hs == 44:
                    flags |= 8
                    d["sec_va"] = (bs(w[14]) << 32) | bs(w[15])
                    d["sec_rkey"], d["sec_len"] = bs(w[16]), bs(w[17])
            d["pkey"] = ((w7 >> 16) & 0xFF) << 8 | (w7 >> 24)
            d["opcode"], d["tran_type"], d["flags"], d["pad_cnt"] = op, tran, flags, pad
    d["status"] = status
    return d


def make_packets(rng):
    """Packets of every opcode the writer knows, plus corrupted opcode / transport / length."""
    pkts = []
    for opcode in (0x06, 0x07, 0x08, 0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x0E, 0x0F, 0x10, 0x11):
        for plen in (0, 1, 2, 3, 4, 77, 256):
            m = oracle.RdmaMsg()
            payload = rng.integers(0, 256, max(plen, 1), dtype=np.uint8)
            m.kind = 1 if opcode == 0x11 else 0
            m.opcode = opcode
            m.tran_type = int(rng.integers(0, 7))
            m.solicited = int(rng.integers(0, 2))
            m.ack_req = int(rng.integers(0, 2))
            m.pkey = int(rng.integers(0, 1 << 16))
            m.dqpn = int(rng.integers(0, 1 << 24))
            m.psn = int(rng.integers(0, 1 << 24))
            m.msn = int(rng.integers(0, 1 << 24))
            m.aeth_code = int(rng.integers(0, 4))
            m.aeth_value = int(rng.integers(0, 32))
            m.reth_va = int(rng.integers(0, 1 << 63))
            m.reth_rkey = int(rng.integers(0, 1 << 32))
            m.reth_len = int(rng.integers(0, 1 << 32))
            m.has_imm = 1
            m.imm = int(rng.integers(0, 1 << 32))
            m.has_secondary_reth = 1
            m.sec_va = int(rng.integers(0, 1 << 63))
            m.sec_rkey = int(rng.integers(0, 1 << 32))
            m.sec_len = int(rng.integers(0, 1 << 32))
            m.payload = payload.ctypes.data
            m.payload_len = plen if opcode not in (0x0C, 0x11) else 0
            rc, pkt = oracle.packet_write(m, 0xC0A80002, 4791, 0xC0A80003, 4791, 1)
            assert rc == 0, (opcode, plen, rc)
            pkts.append(pkt)
    base = pkts[6]  # RDMA WRITE FIRST, 256-byte payload
    bad = base.copy(); bad[28] = (bad[28] & 0xE0) | 0x05; pkts.append(bad)        # SendOnly: invalid opcode
    bad = base.copy(); bad[28] = (7 << 5) | (bad[28] & 0x1F); pkts.append(bad)     # tran_type 7
    bad = base.copy(); bad[29] |= 0x60; pkts.append(bad[:60].copy())               # pad 3, truncated
    rdreq = pkts[7 * 6]                                                             # READ REQUEST (hs 44)
    pkts.append(rdreq[:60].copy())                                                  # header cut short
    bad = base.copy(); bad[100] ^= 1; pkts.append(bad)                              # ICRC mismatch
    pkts.append(base[:43].copy())                                                   # L < 44
    pkts.append(base[:44].copy())
    return pkts


# ---- the reference's own receive-parse expectations (rust_driver/.../tests/test_packet.rs:16-185) ----
def reference_cases():
    """tests/golden/rx_reference_cases.json (made by tests/golden/make_rx_reference.py): four
    IPv4 packets and the fields test_packet.rs asserts `to_rdma_message` decodes from them."""
    import json
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rx_reference_cases.json")
    with open(path) as f:
        cases = json.load(f)
    return [(c["name"], np.frombuffer(bytes.fromhex(c["packet"]), np.uint8), c["expect"]) for c in cases]


def check_reference_expect(d, expect: dict, name: str = "") -> None:
    """One descriptor (oracle.RX_DESC_DTYPE / icrc_rx_desc) against a test_packet.rs case."""
    assert int(d["status"]) == 0 and int(d["icrc_ok"]) == 1, name
    fl = int(d["flags"])
    assert bool(fl & 0x10) == (expect["kind"] == "acknowledge"), name   # Metadata::Acknowledge / General
    assert bool(fl & 0x01) == bool(expect["solicited"]), name
    assert bool(fl & 0x02) == bool(expect["ack_req"]), name
    assert bool(fl & 0x04) == ("imm" in expect), name                    # header.imm is Some
    assert bool(fl & 0x08) == ("sec_va" in expect), name                 # secondary_reth is Some
    for k, v in expect.items():
        if k in ("kind", "solicited", "ack_req"):
            continue
        assert int(d[k]) == int(v), (name, k, int(d[k]), v)
