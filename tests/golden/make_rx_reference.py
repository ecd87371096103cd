"""Generate tests/golden/rx_reference_cases.json — the receive-parse cases the REFERENCE's own
tests pin: rust_driver/src/device/software/tests/test_packet.rs:16-185.

Each reference test fills a zeroed buffer through the packet.rs setters (BTH 97-150, RETH
188-198, AETH 232-241, Immediate 250-252) and asserts what `PacketProcessor::to_rdma_message`
decodes from it.  The header bytes below come from a restatement of those setters (each cites
its line); the EXPECTED fields are the reference's own `assert_eq!` values, copied as data,
with the test_packet.rs line of each.

The receive parse takes whole IPv4 datagrams (include/icrc.h, icrc_rx_parse_device), so each
buffer is wrapped as the emulator's wire form: write_ip_udp_header (packet_processor.rs:307-332;
192.168.0.2 -> 192.168.0.3, port 4791, ip_id 1) in front, the ICRC (zlib CRC-32/ISO-HDLC with
the packet_processor.rs:275-301 masking, independent of the C oracle) as the trailer.  The
reference's buffers carry no trailer, so its payload length (buf_size - header) equals ours
(L - 28 - header - pad - 4).

Run from the repo root:  python tests/golden/make_rx_reference.py
"""
import json
import os
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
MASK = (1, 8, 10, 11, 26, 27, 32)

# ToHostWorkRbDescOpcode (rust_driver/src/device/types.rs:418-429), TransType RC = 0
WRITE_FIRST, WRITE_LAST_IMM, READ_REQUEST, ACKNOWLEDGE = 0x06, 0x09, 0x0C, 0x11
RC = 0


class Bth:
    """packet.rs:37-44 layout, setters 97-150 (on a 12-byte bytearray view)."""

    def __init__(self, b: bytearray, o: int):
        self.b, self.o = b, o

    def set_opcode_and_type(self, opcode, tran):            # packet.rs:97-99
        self.b[self.o] = ((tran << 5) | opcode) & 0xFF

    def set_flags_solicited(self, s):                         # 101-107
        if s:
            self.b[self.o + 1] |= 0x80
        else:
            self.b[self.o + 1] &= 0x7F

    def set_pkey(self, pkey):                                 # 114-116
        self.b[self.o + 2: self.o + 4] = pkey.to_bytes(2, "big")

    def set_destination_qpn(self, qpn):                       # 118-120
        self.b[self.o + 4: self.o + 8] = (qpn & 0xFFFFFF).to_bytes(4, "big")

    def set_ack_req(self, a):                                 # 122-128
        if a:
            self.b[self.o + 8] |= 0x80
        else:
            self.b[self.o + 8] &= 0x7F

    def set_psn(self, psn):                                   # 130-134: keeps byte 0 (ack_req)
        keep = self.b[self.o + 8]
        self.b[self.o + 8: self.o + 12] = (psn & 0xFFFFFF).to_bytes(4, "big")
        self.b[self.o + 8] = keep


def set_reth(b: bytearray, o: int, va: int, rkey: int, dlen: int):  # packet.rs:188-198
    b[o: o + 8] = va.to_bytes(8, "big")
    b[o + 8: o + 12] = rkey.to_bytes(4, "big")
    b[o + 12: o + 16] = dlen.to_bytes(4, "big")


def set_aeth(b: bytearray, o: int, code: int, value: int, msn: int):  # packet.rs:232-241
    b[o] = (((code % 4) << 5) | value) & 0xFF
    keep = b[o]
    b[o: o + 4] = (msn & 0xFFFFFF).to_bytes(4, "big")
    b[o] = keep


def bth_common(buf, opcode, pkey):
    """The BTH setter sequence every test_packet.rs case runs (e.g. :19-25)."""
    bth = Bth(buf, 0)
    bth.set_opcode_and_type(opcode, RC)
    bth.set_destination_qpn(1)
    bth.set_psn(1)
    bth.set_ack_req(False)
    bth.set_flags_solicited(True)
    bth.set_pkey(pkey)


def wrap(udp_payload: bytes) -> bytes:
    """write_ip_udp_header (packet_processor.rs:307-332) + payload + ICRC trailer."""
    L = 28 + len(udp_payload) + 4
    ip = bytes([0x45, 0, *L.to_bytes(2, "big"), 0, 1, 0, 0, 64, 17, 0, 0, 192, 168, 0, 2, 192, 168, 0, 3])
    udp = (4791).to_bytes(2, "big") * 2 + (L - 20).to_bytes(2, "big") + b"\0\0"
    body = ip + udp + udp_payload
    h = bytearray(body[:40])
    for o in MASK:
        h[o] = 0xFF
    icrc = zlib.crc32(b"\xff" * 8 + bytes(h) + body[40:])
    return body + icrc.to_bytes(4, "little")


def cases():
    out = []
    # test_header_bth_reth (test_packet.rs:16-55): BTH + RETH + 512 zero bytes
    b = bytearray(12 + 16 + 512)
    bth_common(b, WRITE_FIRST, 0x1234)
    set_reth(b, 12, 1, 0x12345678, 1)
    out.append(dict(name="test_header_bth_reth", ref="test_packet.rs:16-55", packet=wrap(bytes(b)).hex(),
                    expect=dict(tran_type=RC, opcode=WRITE_FIRST, solicited=1, dqpn=1, ack_req=0, psn=1,
                                pkey=0x1234, reth_va=1, reth_rkey=0x12345678, reth_len=1, payload_len=512,
                                kind="general")))
    # test_header_bth_reth_imm (:57-103): BTH + RETH + Imm [1,1,1,1] + 512
    b = bytearray(12 + 16 + 4 + 512)
    bth_common(b, WRITE_LAST_IMM, 0x1234)
    set_reth(b, 12, 0x1234567812345678, 0x12345678, 0x12345678)
    b[28:32] = bytes([1, 1, 1, 1])
    out.append(dict(name="test_header_bth_reth_imm", ref="test_packet.rs:57-103", packet=wrap(bytes(b)).hex(),
                    expect=dict(tran_type=RC, opcode=WRITE_LAST_IMM, solicited=1, dqpn=1, ack_req=0, psn=1,
                                pkey=0x1234, reth_va=0x1234567812345678, reth_rkey=0x12345678,
                                reth_len=0x12345678, payload_len=512, imm=0x01010101, kind="general")))
    # test_header_bth_reth_reth (:105-152): BTH + RETH + secondary RETH, no payload
    b = bytearray(12 + 16 + 16)
    bth_common(b, READ_REQUEST, 0x1234)
    set_reth(b, 12, 0x1234567812345678, 0x12345678, 0x12345678)
    set_reth(b, 28, 0x1234567812345678, 0x12345678, 0x12345678)
    out.append(dict(name="test_header_bth_reth_reth", ref="test_packet.rs:105-152", packet=wrap(bytes(b)).hex(),
                    expect=dict(tran_type=RC, opcode=READ_REQUEST, solicited=1, dqpn=1, ack_req=0, psn=1,
                                pkey=0x1234, reth_va=0x1234567812345678, reth_rkey=0x12345678,
                                reth_len=0x12345678, payload_len=0, sec_va=0x1234567812345678,
                                sec_rkey=0x12345678, sec_len=0x12345678, kind="general")))
    # test_header_bth_aeth (:154-185): BTH + AETH {code 2, value 5, msn 0x123456}
    b = bytearray(12 + 4)
    bth_common(b, ACKNOWLEDGE, 1)
    set_aeth(b, 12, 2, 5, 0x123456)  # set_aeth_code_and_value(2, 5), then set_msn (keeps byte 0)
    out.append(dict(name="test_header_bth_aeth", ref="test_packet.rs:154-185", packet=wrap(bytes(b)).hex(),
                    expect=dict(tran_type=RC, opcode=ACKNOWLEDGE, solicited=1, dqpn=1, ack_req=0, psn=1,
                                aeth_msn=0x123456, aeth_code=2, aeth_value=5, kind="acknowledge")))
    return out


def main():
    path = os.path.join(HERE, "rx_reference_cases.json")
    with open(path, "w") as f:
        json.dump(cases(), f, indent=1)
        f.write("\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
