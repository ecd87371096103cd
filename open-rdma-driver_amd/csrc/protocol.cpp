// protocol.cpp — product-side packet serialisation (the PacketWriter half of the surface).
//
// Mirrors blue-rdma-device/src/third_party/net/packet_processor.rs:150-265 (PacketWriter),
// 303-332 (write_ip_udp_header) and the header setters of packet.rs:100-243, 458-515.
// Header bytes are host work (a few dozen stores); the ICRC itself is always the GPU
// kernel, reached through icrc_compute().
#include <cstring>

#include "icrc.h"

namespace {

inline void be16(uint8_t *p, uint16_t v) {
    p[0] = uint8_t(v >> 8);
    p[1] = uint8_t(v);
}
inline void be32(uint8_t *p, uint32_t v) {
    p[0] = uint8_t(v >> 24);
    p[1] = uint8_t(v >> 16);
    p[2] = uint8_t(v >> 8);
    p[3] = uint8_t(v);
}
inline void be64(uint8_t *p, uint64_t v) {
    be32(p, uint32_t(v >> 32));
    be32(p + 4, uint32_t(v));
}

// PayloadInfo::get_pad_cnt (types.rs:155-162)
inline uint32_t pad_cnt(uint64_t len) { return uint32_t((4u - len % 4u) % 4u); }

// BTH::set_from_common_meta (packet.rs:145-153): the same read-modify-write sequence.
void set_bth(uint8_t *bth, const icrc_rdma_msg &m, uint32_t pad) {
    bth[0] = uint8_t(uint8_t(m.tran_type << 5) | m.opcode);
    bth[1] = m.solicited ? uint8_t(bth[1] | 0x80u) : uint8_t(bth[1] & 0x7fu);
    bth[1] = uint8_t((bth[1] & 0x9fu) | uint8_t(pad << 5));
    be32(bth + 4, m.dqpn & 0x00ffffffu);
    bth[8] = m.ack_req ? uint8_t(bth[8] | 0x80u) : uint8_t(bth[8] & 0x7fu);
    const uint8_t ack = bth[8];
    be32(bth + 8, m.psn & 0x00ffffffu);
    bth[8] = ack;
    be16(bth + 2, m.pkey);
}

// PacketProcessor::set_from_rdma_message (packet_processor.rs:73-124; packet.rs:304-424).
int set_rdma_header(uint8_t *h, const icrc_rdma_msg &m) {
    const int hl = icrc_rdma_header_len(m.opcode);
    if (hl < 0) return hl;
    const uint32_t pad = pad_cnt(m.payload_len);
    if (m.opcode == 0x11) {  // Acknowledge: RdmaHeaderRespBthAeth
        if (m.kind != 1) return ICRC_EINVALID_METADATA;
        set_bth(h, m, pad);
        h[12] = uint8_t(((m.aeth_code % 4u) << 5) | m.aeth_value);
        const uint8_t v0 = h[12];
        be32(h + 12, m.msn & 0x00ffffffu);
        h[12] = v0;
        return hl;
    }
    if (m.kind != 0) return ICRC_EINVALID_METADATA;
    set_bth(h, m, pad);
    be64(h + 12, m.reth_va);
    be32(h + 20, m.reth_rkey);
    be32(h + 24, m.reth_len);
    if (hl == 32) {
        if (!m.has_imm) return ICRC_EINVALID_METADATA;
        be32(h + 28, m.imm);
    } else if (hl == 44) {
        if (!m.has_secondary_reth) return ICRC_EINVALID_METADATA;
        be64(h + 28, m.sec_va);
        be32(h + 36, m.sec_rkey);
        be32(h + 40, m.sec_len);
    }
    return hl;
}

int plan(const icrc_rdma_msg *msg, int *hl, uint64_t *total) {
    if (!msg) return ICRC_EINVAL;
    *hl = icrc_rdma_header_len(msg->opcode);
    if (*hl < 0) return *hl;
    *total = 28u + uint64_t(*hl) + msg->payload_len + pad_cnt(msg->payload_len) + 4u;
    if (*total > 0xffffu) return ICRC_ELENGTH_TOO_LONG;
    return ICRC_OK;
}

}  // namespace

extern "C" {

int icrc_rdma_header_len(uint8_t opcode) {
    switch (opcode) {
    case 0x06: case 0x07: case 0x08: case 0x0a:
    case 0x0d: case 0x0e: case 0x0f: case 0x10: return 28;
    case 0x09: case 0x0b: return 32;
    case 0x0c: return 44;
    case 0x11: return 16;
    default: return ICRC_EINVALID_OPCODE;
    }
}

void icrc_write_ip_udp_header(uint8_t *buf, uint32_t src_ip, uint16_t src_port, uint32_t dst_ip,
                              uint16_t dst_port, uint16_t total_length, uint16_t ip_id) {
    buf[0] = 0x45;  // Ipv4Header::set_default_header (packet.rs:458-463)
    buf[1] = 0x00;
    buf[8] = 64;
    buf[9] = 0x11;
    be32(buf + 12, src_ip);
    be32(buf + 16, dst_ip);
    be16(buf + 2, total_length);
    be16(buf + 6, 0);
    be16(buf + 4, ip_id);
    be16(buf + 10, 0);
    be16(buf + 20, src_port);
    be16(buf + 22, dst_port);
    be16(buf + 24, uint16_t(total_length - 20));
    be16(buf + 26, 0);
}

int icrc_packet_headers(uint8_t *buf, size_t buf_len, const icrc_rdma_msg *msg, uint32_t src_ip,
                        uint16_t src_port, uint32_t dst_ip, uint16_t dst_port, uint16_t ip_id,
                        size_t *out_hdr_len, size_t *out_total_len) {
    if (!buf) return ICRC_EINVAL;
    if (buf_len < 28) return ICRC_EBUFFER_NOT_LARGE;
    int hl;
    uint64_t total;
    int rc = plan(msg, &hl, &total);
    if (rc) return rc;
    if (buf_len < size_t(28 + hl)) return ICRC_EBUFFER_NOT_LARGE;
    rc = set_rdma_header(buf + 28, *msg);
    if (rc < 0) return rc;
    icrc_write_ip_udp_header(buf, src_ip, src_port, dst_ip, dst_port, uint16_t(total), ip_id);
    if (out_hdr_len) *out_hdr_len = size_t(28 + hl);
    if (out_total_len) *out_total_len = size_t(total);
    return ICRC_OK;
}

int icrc_packet_write(uint8_t *buf, size_t buf_len, const icrc_rdma_msg *msg, uint32_t src_ip,
                      uint16_t src_port, uint32_t dst_ip, uint16_t dst_port, uint16_t ip_id,
                      size_t *out_len) {
    if (!buf) return ICRC_EINVAL;
    if (buf_len < 28) return ICRC_EBUFFER_NOT_LARGE;
    int hl;
    uint64_t total;
    int rc = plan(msg, &hl, &total);
    if (rc) return rc;
    if (buf_len < total) return ICRC_EBUFFER_NOT_LARGE;  // checked before any write
    rc = set_rdma_header(buf + 28, *msg);
    if (rc < 0) return rc;
    if (msg->payload_len) std::memcpy(buf + 28 + hl, msg->payload, msg->payload_len);
    icrc_write_ip_udp_header(buf, src_ip, src_port, dst_ip, dst_port, uint16_t(total), ip_id);
    int err = ICRC_OK;
    const uint32_t c = icrc_compute(buf, size_t(total), &err);
    if (err) return err;
    buf[total - 4] = uint8_t(c);
    buf[total - 3] = uint8_t(c >> 8);
    buf[total - 2] = uint8_t(c >> 16);
    buf[total - 1] = uint8_t(c >> 24);
    if (out_len) *out_len = size_t(total);
    return ICRC_OK;
}

}  // extern "C"
