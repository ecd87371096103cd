/*
 * oracle/icrc_oracle.c — TEST INFRASTRUCTURE ONLY.  See icrc_oracle.h for the contract.
 *
 * A plain-C restatement of the reference ICRC path, written for clarity, not speed.
 * Every function cites the reference file:line it follows (paths relative to the
 * reference root, blue-rdma-device/src/ unless stated).  Nothing in the product
 * (open-rdma-driver_amd/) links or calls this file.
 */
#include "icrc_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------- */
/* CRC-32/ISO-HDLC, as crc32fast 1.4.2 computes it (Cargo.lock:230-236).              */
/* crc32fast::Hasher::update(buf): state = !update(!state, buf) with the reflected    */
/* polynomial 0xEDB88320; Hasher::new() starts at state 0; finalize() returns state.   */
/* That is zlib's crc32(crc, buf, len) chaining convention.                           */
/* ---------------------------------------------------------------------------------- */
static uint32_t crc_table[256];
static int crc_table_ready;

static void crc_table_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        crc_table[i] = c;
    }
    __atomic_store_n(&crc_table_ready, 1, __ATOMIC_RELEASE);
}

uint32_t oracle_crc32(uint32_t crc, const uint8_t *p, size_t n) {
    if (!__atomic_load_n(&crc_table_ready, __ATOMIC_ACQUIRE)) crc_table_init();
    crc = ~crc;
    for (size_t i = 0; i < n; i++) crc = crc_table[(crc ^ p[i]) & 0xffu] ^ (crc >> 8);
    return ~crc;
}

/* ---------------------------------------------------------------------------------- */
/* compute_icrc — third_party/net/packet_processor.rs:275-301                          */
/*   hasher.update([0xff; 8])                                   (277-278)              */
/*   copy CommonPacketHeader (40 B = IPv4 20 + UDP 8 + BTH 12)  (280, packet.rs:538)   */
/*   ip.dscp_ecn = 0xff  -> byte 1                              (282, packet.rs:445)   */
/*   ip.ttl = 0xff       -> byte 8                              (283, packet.rs:449)   */
/*   ip.checksum = 0xffff -> bytes 10..11                       (284, packet.rs:451)   */
/*   udp.checksum = 0xffff -> bytes 26..27                      (285, packet.rs:497)   */
/*   bth.fill_ecn_and_resv6 -> destination_qpn[0] = byte 32     (286, packet.rs:140)   */
/*   hasher.update(hdr40); hasher.update(data[40 .. len-4])     (296-298)              */
/* The reference panics for len < 44 (slice at 298); here that is -EINVAL.             */
/* ---------------------------------------------------------------------------------- */
int oracle_compute_icrc(const uint8_t *pkt, size_t len, uint32_t *out) {
    if (pkt == NULL || out == NULL || len < 44) return ORACLE_EINVAL;
    static const uint8_t prefix[8] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    uint8_t hdr[40];
    memcpy(hdr, pkt, 40);
    hdr[1] = 0xff;
    hdr[8] = 0xff;
    hdr[10] = 0xff;
    hdr[11] = 0xff;
    hdr[26] = 0xff;
    hdr[27] = 0xff;
    hdr[32] = 0xff;
    uint32_t crc = oracle_crc32(0, prefix, 8);
    crc = oracle_crc32(crc, hdr, 40);
    crc = oracle_crc32(crc, pkt + 40, len - 44);
    *out = crc;
    return ORACLE_OK;
}

/* is_icrc_valid — packet_processor.rs:341-353: read trailer LE (344-349), zero it in   */
/* place (350), recompute (351), compare (352).                                         */
int oracle_is_icrc_valid(uint8_t *pkt, size_t len, int *ok) {
    if (pkt == NULL || ok == NULL || len < 44) return ORACLE_EINVAL;
    uint32_t origin = (uint32_t)pkt[len - 4] | ((uint32_t)pkt[len - 3] << 8) |
                      ((uint32_t)pkt[len - 2] << 16) | ((uint32_t)pkt[len - 1] << 24);
    memset(pkt + len - 4, 0, 4);
    uint32_t ours;
    int rc = oracle_compute_icrc(pkt, len, &ours);
    if (rc) return rc;
    *ok = (ours == origin);
    return ORACLE_OK;
}

int oracle_compute_icrc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                              uint64_t n, uint32_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        int rc = oracle_compute_icrc(base + off[i], len[i], &out[i]);
        if (rc) return rc;
    }
    return ORACLE_OK;
}

/* ---------------------------------------------------------------------------------- */
/* Header serialisation                                                                */
/* ---------------------------------------------------------------------------------- */
static void put_be16(uint8_t *p, uint16_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
static void put_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}
static void put_be64(uint8_t *p, uint64_t v) {
    put_be32(p, (uint32_t)(v >> 32));
    put_be32(p + 4, (uint32_t)v);
}

/* write_ip_udp_header — packet_processor.rs:307-332 with the setters of packet.rs:458-515.
 * ip/udp addresses are given in host order (a.b.c.d = a<<24|b<<16|c<<8|d). */
void oracle_write_ip_udp_header(uint8_t *buf, uint32_t src_ip, uint16_t src_port, uint32_t dst_ip,
                                uint16_t dst_port, uint16_t total_length, uint16_t ip_id) {
    buf[0] = 0x45; /* set_default_header, packet.rs:458-463 */
    buf[1] = 0x00;
    buf[8] = 64;
    buf[9] = 0x11;
    put_be32(buf + 12, src_ip);       /* set_source 481 */
    put_be32(buf + 16, dst_ip);       /* set_destination 485 */
    put_be16(buf + 2, total_length);  /* set_total_length 465 */
    put_be16(buf + 6, 0);             /* set_flags_fragment_offset 473 */
    put_be16(buf + 4, ip_id);         /* set_identification 469 */
    put_be16(buf + 10, 0);            /* set_checksum 477 */
    put_be16(buf + 20, src_port);     /* udp set_source_port 501 */
    put_be16(buf + 22, dst_port);     /* set_dest_port 505 */
    put_be16(buf + 24, (uint16_t)(total_length - 20)); /* set_length 509, 330 */
    put_be16(buf + 26, 0);            /* set_checksum 513 */
}

/* Header composite sizes per opcode — packet.rs:427-438. */
int oracle_header_len(uint8_t opcode) {
    switch (opcode) {
    case OP_WRITE_FIRST:
    case OP_WRITE_MIDDLE:
    case OP_WRITE_LAST:
    case OP_WRITE_ONLY:
    case OP_READ_RESP_FIRST:
    case OP_READ_RESP_MIDDLE:
    case OP_READ_RESP_LAST:
    case OP_READ_RESP_ONLY: return 28; /* RdmaHeaderReqBthReth */
    case OP_WRITE_LAST_IMM:
    case OP_WRITE_ONLY_IMM: return 32; /* RdmaHeaderReqBthRethImm */
    case OP_READ_REQUEST: return 44;   /* RdmaHeaderReqBthDoubleReth */
    case OP_ACK: return 16;            /* RdmaHeaderRespBthAeth */
    default: return ORACLE_INVALID_OPCODE;
    }
}

/* PayloadInfo::get_pad_cnt — types.rs:155-162 */
uint32_t oracle_pad_cnt(uint64_t payload_len) {
    uint32_t pad = 4u - (uint32_t)(payload_len % 4u);
    return pad == 4u ? 0u : pad;
}

/* BTH::set_from_common_meta — packet.rs:145-153, each setter read-modify-writes the
 * caller's buffer exactly like the reference (100-137). */
static void bth_set_from_common_meta(uint8_t *bth, const oracle_rdma_msg *m, uint32_t pad_cnt) {
    bth[0] = (uint8_t)((uint8_t)(m->tran_type << 5) | m->opcode);        /* 100-102 */
    if (m->solicited) bth[1] |= 0x80; else bth[1] &= (uint8_t)~0x80u;     /* 104-110 */
    bth[1] = (uint8_t)((bth[1] & (uint8_t)~0x60u) | (uint8_t)(pad_cnt << 5)); /* 113-115 */
    put_be32(bth + 4, m->dqpn & 0x00FFFFFFu);                            /* 121-123 */
    if (m->ack_req) bth[8] |= 0x80; else bth[8] &= (uint8_t)~0x80u;      /* 125-131 */
    {                                                                     /* 133-137 */
        uint8_t ack = bth[8];
        put_be32(bth + 8, m->psn & 0x00FFFFFFu);
        bth[8] = ack;
    }
    put_be16(bth + 2, m->pkey);                                           /* 117-119 */
}

/* PacketProcessor::set_from_rdma_message — packet_processor.rs:73-124 and the header
 * impls packet.rs:304-424.  Returns the header length or an error. */
static int set_from_rdma_message(uint8_t *h, const oracle_rdma_msg *m) {
    int hl = oracle_header_len(m->opcode);
    if (hl < 0) return hl;
    uint32_t pad = oracle_pad_cnt(m->payload_len);
    if (m->opcode == OP_ACK) {
        if (m->kind != 1) return ORACLE_INVALID_METADATA; /* 422 */
        bth_set_from_common_meta(h, m, pad);
        h[12] = (uint8_t)(((m->aeth_code % 4u) << 5) | m->aeth_value); /* 234-236 */
        {
            uint8_t v0 = h[12]; /* set_msn 238-242 */
            put_be32(h + 12, m->msn & 0x00FFFFFFu);
            h[12] = v0;
        }
        return hl;
    }
    if (m->kind != 0) return ORACLE_INVALID_METADATA; /* 312, 351, 389 */
    bth_set_from_common_meta(h, m, pad);
    put_be64(h + 12, m->reth_va); /* RETH::set_from_reth_header 197-201 */
    put_be32(h + 20, m->reth_rkey);
    put_be32(h + 24, m->reth_len);
    if (hl == 32) {
        if (!m->has_imm) return ORACLE_INVALID_METADATA; /* 386 */
        put_be32(h + 28, m->imm);
    } else if (hl == 44) {
        if (!m->has_secondary_reth) return ORACLE_INVALID_METADATA; /* 347 */
        put_be64(h + 28, m->sec_va);
        put_be32(h + 36, m->sec_rkey);
        put_be32(h + 40, m->sec_len);
    }
    return hl;
}

/* PacketWriter::write — packet_processor.rs:210-265.  All builder fields are supplied.
 * Unlike the reference (whose header/payload writes are unchecked raw-pointer writes that
 * precede the final length check at 253-256) the buffer size is checked before any write. */
int oracle_packet_write(uint8_t *buf, size_t buf_len, const oracle_rdma_msg *msg, uint32_t src_ip,
                        uint16_t src_port, uint32_t dst_ip, uint16_t dst_port, uint16_t ip_id,
                        size_t *out_len) {
    if (msg == NULL) return ORACLE_EINVAL;
    if (buf_len < 28) return ORACLE_BUFFER_NOT_LARGE; /* 215-218 */
    int hl = oracle_header_len(msg->opcode);
    if (hl < 0) return hl;
    uint64_t padded = msg->payload_len + oracle_pad_cnt(msg->payload_len); /* types.rs:164 */
    uint64_t total = 28u + (uint64_t)hl + padded + 4u;                      /* 222-225 */
    if (total > 0xFFFFu) return ORACLE_LENGTH_TOO_LONG;                     /* 226-227 */
    if (buf_len < total) return ORACLE_BUFFER_NOT_LARGE;                    /* 253-256 */
    int rc = set_from_rdma_message(buf + 28, msg);                           /* 219 */
    if (rc < 0) return rc;
    if (msg->payload_len) memcpy(buf + 28 + hl, msg->payload, msg->payload_len); /* 235 */
    oracle_write_ip_udp_header(buf, src_ip, src_port, dst_ip, dst_port, (uint16_t)total, ip_id);
    uint32_t icrc;
    rc = oracle_compute_icrc(buf, total, &icrc); /* 260 */
    if (rc) return rc;
    buf[total - 4] = (uint8_t)icrc; /* to_le_bytes, 260-263 */
    buf[total - 3] = (uint8_t)(icrc >> 8);
    buf[total - 2] = (uint8_t)(icrc >> 16);
    buf[total - 1] = (uint8_t)(icrc >> 24);
    if (out_len) *out_len = (size_t)total;
    return ORACLE_OK;
}

/* generate_ack — net/util.rs:134-170: BTH(ACK, RC, dqpn=peer_qpn, psn=expected_psn,
 * ack_req=0, solicited=0, pkey) + AETH(code Ack, value 0x1f, msn = pkey), written by
 * PacketWriter from 192.168.0.3 to 192.168.0.2, port 4791, ip_id 1, into a 48-B buffer. */
int oracle_generate_ack(uint16_t pkey, uint32_t peer_qpn, uint32_t expected_psn, uint8_t *pkt48,
                        uint8_t *udp_payload20) {
    oracle_rdma_msg m;
    memset(&m, 0, sizeof m);
    m.kind = 1;
    m.opcode = OP_ACK;
    m.tran_type = 0;
    m.pkey = pkey;
    m.dqpn = peer_qpn;
    m.psn = expected_psn;
    m.aeth_code = 0;
    m.aeth_value = 0x1f;
    m.msn = pkey; /* util.rs:150 */
    uint8_t buf[48];
    memset(buf, 0, sizeof buf);
    size_t len = 0;
    int rc = oracle_packet_write(buf, sizeof buf, &m, 0xC0A80003u, 4791, 0xC0A80002u, 4791, 1, &len);
    if (rc) return rc;
    if (len != 48) return ORACLE_EINVAL; /* util.rs:166 */
    if (pkt48) memcpy(pkt48, buf, 48);
    if (udp_payload20) memcpy(udp_payload20, buf + 28, 20); /* util.rs:167-169 */
    return ORACLE_OK;
}

/* generate_segments_from_request — queues/send/operations/common.rs:152-176 */
uint32_t oracle_generate_segments(uint64_t va, uint32_t len, uint32_t path_mtu, uint64_t *seg_va,
                                  uint32_t *seg_len, uint32_t max_segs) {
    uint32_t n = 0;
    uint32_t remainder = len;
    uint32_t first = path_mtu - ((uint32_t)va % path_mtu);
    if (remainder < first) first = remainder;
    if (n < max_segs) {
        seg_va[n] = va;
        seg_len[n] = first;
    }
    n++;
    va += first;
    remainder -= first;
    while (remainder > 0) {
        uint32_t l = remainder < path_mtu ? remainder : path_mtu;
        if (n < max_segs) {
            seg_va[n] = va;
            seg_len[n] = l;
        }
        n++;
        va += l;
        remainder -= l;
    }
    return n;
}

/* ---- rust_driver's send rule: BlueRDMALogic::send (rust_driver/src/device/software/logic.rs) ---- */

/* ToHostWorkRbDescOpcode::is_first — rust_driver/src/device/types.rs:433-447 */
static int opcode_is_first(uint8_t op) { return op == OP_WRITE_FIRST || op == OP_READ_RESP_FIRST; }

/* get_first_packet_max_length — rust_driver/src/utils.rs:19-25 */
static uint32_t first_packet_max_length(uint64_t va, uint32_t pmtu) { return pmtu - (uint32_t)(va % pmtu); }

/* ToCardWriteDescriptor::write_only_opcode_with_imm — types.rs:558-581 */
static uint8_t write_only_opcode_with_imm(const oracle_write_desc *d, int *with_imm) {
    *with_imm = 0;
    if (d->is_first && d->is_last) {
        if (d->is_resp) return OP_READ_RESP_ONLY;
        if (d->has_imm) { *with_imm = 1; return OP_WRITE_ONLY_IMM; }
        return OP_WRITE_ONLY;
    } else if (d->is_first) {
        return d->is_resp ? OP_READ_RESP_FIRST : OP_WRITE_FIRST;
    } else { /* "self.is_last = True" (also reached with is_last false) */
        if (d->is_resp) return OP_READ_RESP_LAST;
        if (d->has_imm) { *with_imm = 1; return OP_WRITE_LAST_IMM; }
        return OP_WRITE_LAST;
    }
}

/* write_first_opcode — types.rs:583-590 */
static uint8_t write_first_opcode(const oracle_write_desc *d) {
    if (d->is_first) return d->is_resp ? OP_READ_RESP_FIRST : OP_WRITE_FIRST;
    return d->is_resp ? OP_READ_RESP_MIDDLE : OP_WRITE_MIDDLE;
}

/* write_middle_opcode — types.rs:592-598 */
static uint8_t write_middle_opcode(const oracle_write_desc *d) {
    return d->is_resp ? OP_READ_RESP_MIDDLE : OP_WRITE_MIDDLE;
}

/* write_last_opcode_with_imm — types.rs:600-609 */
static uint8_t write_last_opcode_with_imm(const oracle_write_desc *d, int *with_imm) {
    *with_imm = 0;
    if (d->is_last) {
        if (d->is_resp) return OP_READ_RESP_LAST;
        if (d->has_imm) { *with_imm = 1; return OP_WRITE_LAST_IMM; }
        return OP_WRITE_LAST;
    }
    return d->is_resp ? OP_READ_RESP_MIDDLE : OP_WRITE_MIDDLE;
}

static void logic_emit(oracle_logic_pkt *out, uint32_t max_out, uint32_t *n, uint8_t op, int with_imm,
                       uint32_t imm, uint32_t psn, uint64_t va, uint32_t reth_len, uint32_t off, uint32_t len) {
    if (*n < max_out) {
        oracle_logic_pkt *p = &out[*n];
        memset(p, 0, sizeof *p);
        p->opcode = op;
        p->has_imm = (uint8_t)(with_imm != 0);
        p->imm = with_imm ? imm : 0u;
        p->psn = psn & 0x00FFFFFFu;
        p->reth_va = va;
        p->reth_len = reth_len;
        p->payload_off = off;
        p->payload_len = len;
    }
    (*n)++;
}

/* BlueRDMALogic::send for ToCardDescriptor::Write — logic.rs:191-271, with
 * send_write_only_packet (109-134).  Psn::wrapping_add is mod 2^24 (rust_driver/src/types.rs:180-183). */
uint32_t oracle_logic_send(const oracle_write_desc *d, oracle_logic_pkt *out, uint32_t max_out) {
    uint32_t n = 0;
    if (d == NULL || d->pmtu == 0) return 0;
    const uint32_t pmtu = d->pmtu;                                               /* 193 */
    const uint32_t first_max = first_packet_max_length(d->raddr, pmtu);           /* 194 */
    const uint32_t sge_total = d->sge_len;                                        /* 207 */
    int with_imm = 0;
    if (sge_total <= first_max) {                                                 /* 208-210 */
        /* send_write_only_packet, 109-134 */
        uint8_t op = write_only_opcode_with_imm(d, &with_imm);                    /* 118 */
        uint32_t reth_len = opcode_is_first(op) ? d->total_len : sge_total;       /* 121-125 */
        logic_emit(out, max_out, &n, op, with_imm, d->imm, d->psn, d->raddr, reth_len, 0, sge_total);
        return n;
    }
    uint64_t cur_va = d->raddr;                                                   /* 214 */
    uint32_t cur_len = sge_total;                                                 /* 215 */
    uint32_t psn = d->psn;                                                        /* 216 */
    uint32_t pos = 0;
    const uint32_t first_len = first_max;                                         /* 220 */
    uint8_t op = write_first_opcode(d);                                           /* 223 */
    uint32_t reth_len = opcode_is_first(op) ? d->total_len : first_len;           /* 224-228 */
    logic_emit(out, max_out, &n, op, 0, 0, psn, cur_va, reth_len, pos, first_len); /* 229-237 */
    cur_len -= first_len;
    psn = (psn + 1u) & 0x00FFFFFFu;
    cur_va += first_len;
    pos += first_len;
    while (cur_len > pmtu) {                                                      /* 240-254 */
        logic_emit(out, max_out, &n, write_middle_opcode(d), 0, 0, psn, cur_va, pmtu, pos, pmtu);
        cur_len -= pmtu;
        psn = (psn + 1u) & 0x00FFFFFFu;
        cur_va += pmtu;
        pos += pmtu;
    }
    op = write_last_opcode_with_imm(d, &with_imm);                                /* 256-270 */
    logic_emit(out, max_out, &n, op, with_imm, d->imm, psn, cur_va, cur_len, pos, cur_len);
    return n;
}

/* calculate_ipv4_checksum — rust_driver/src/responser.rs:321-338 */
uint16_t oracle_ipv4_checksum(const uint8_t *h) {
    uint32_t sum = 0;
    for (int i = 0; i < 20; i += 2) sum += ((uint32_t)h[i] << 8) | h[i + 1];
    while (sum >> 16) sum = (sum & 0xFFFFu) + (sum >> 16);
    return (uint16_t)~sum;
}

/* ---------------------------------------------------------------------------------- */
/* Receive: is_icrc_valid, then to_rdma_message on buf = pkt[28 .. len-4)              */
/* ---------------------------------------------------------------------------------- */
static uint32_t get_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* Header struct size per opcode: PacketProcessor::to_rdma_message's dispatch
 * (packet_processor.rs:18-71) over the layouts of packet.rs:286-438. */
static int rx_header_size(uint8_t opcode) {
    switch (opcode) {
    case 0x06: case 0x07: case 0x08: case 0x0A:        /* RdmaWrite{First,Middle,Last,Only}  */
    case 0x0D: case 0x0E: case 0x0F: case 0x10:        /* RdmaReadResponse*                  */
        return 28;                                     /* RdmaHeaderReqBthReth               */
    case 0x09: case 0x0B: return 32;                   /* RdmaHeaderReqBthRethImm            */
    case 0x0C: return 44;                              /* RdmaHeaderReqBthDoubleReth         */
    case 0x11: return 16;                              /* RdmaHeaderRespBthAeth              */
    default: return -1;                                /* Err(PacketError::InvalidOpcode)    */
    }
}

int oracle_rx_parse(uint8_t *pkt, uint32_t len, uint64_t off, int zero_trailer, oracle_rx_desc *d) {
    memset(d, 0, sizeof *d);
    if (len < 44) {
        d->icrc_ok = 0xFF;
        d->status = 3;
        return ORACLE_OK;
    }
    uint8_t saved[4];
    memcpy(saved, pkt + len - 4, 4);
    int ok = 0;
    oracle_is_icrc_valid(pkt, len, &ok); /* zeroes the trailer (packet_processor.rs:350) */
    if (!zero_trailer) memcpy(pkt + len - 4, saved, 4);
    d->icrc_ok = ok ? 1 : 0;

    const uint8_t *buf = pkt + 28;             /* UDP payload ... */
    const uint32_t buf_size = len - 4 - 28;    /* ... with the ICRC stripped */
    const uint8_t opcode = buf[0] & 0x1F;      /* BTH::get_opcode (packet.rs:61-63) */
    const uint8_t tran = (buf[0] & 0xE0) >> 5; /* get_transaction_type (57-59) */
    const int hs = rx_header_size(opcode);
    if (hs < 0) {
        d->status = 1;
        return ORACLE_OK;
    }
    if (tran > 6) { /* ToHostWorkRbDescTransType::try_from (types.rs:244-245) */
        d->status = 2;
        return ORACLE_OK;
    }
    const uint8_t pad = (buf[1] & 0x60) >> 5; /* get_pad_cnt (69-71) */
    if (buf_size < (uint32_t)hs + pad) {      /* the reference would read past the buffer */
        d->status = 3;
        return ORACLE_OK;
    }
    d->opcode = opcode;
    d->tran_type = tran;
    d->pad_cnt = pad;
    d->flags = (uint8_t)(((buf[1] & 0x80) ? 0x01 : 0) | ((buf[8] & 0x80) ? 0x02 : 0));
    d->pkey = (uint16_t)((buf[2] << 8) | buf[3]);   /* get_pkey (79-81) */
    d->dqpn = get_be32(buf + 4) & 0x00FFFFFFu;       /* get_destination_qpn (83-90) */
    d->psn = get_be32(buf + 8) & 0x00FFFFFFu;        /* get_psn (96-98); get_ack_req (92-94) */
    d->payload_offset = off + 28 + (uint64_t)hs;     /* get_data_ptr (267-269) */
    d->payload_len = buf_size - (uint32_t)hs - pad;  /* get_packet_real_length (74-77) */
    if (opcode == 0x11) {                            /* AethHeader::new_from_packet (types.rs:318-329) */
        d->flags |= 0x10;
        d->aeth_code = (buf[12] & 0x60) >> 5;
        d->aeth_value = buf[12] & 0x1F;
        d->aeth_msn = get_be32(buf + 12) & 0x00FFFFFFu;
        return ORACLE_OK;
    }
    d->reth_va = ((uint64_t)get_be32(buf + 12) << 32) | get_be32(buf + 16); /* RETH getters (173-183) */
    d->reth_rkey = get_be32(buf + 20);
    d->reth_len = get_be32(buf + 24);
    if (hs == 32) {
        d->flags |= 0x04;
        d->imm = get_be32(buf + 28); /* Immediate::get (packet.rs:249-251) */
    } else if (hs == 44) {
        d->flags |= 0x08;
        d->sec_va = ((uint64_t)get_be32(buf + 28) << 32) | get_be32(buf + 32);
        d->sec_rkey = get_be32(buf + 36);
        d->sec_len = get_be32(buf + 40);
    }
    return ORACLE_OK;
}

/* oracle_rx_parse over a ragged batch (packet i at base + off[i], len[i] bytes): the same per-packet
 * restatement, looped here so that a million-packet check costs no per-packet call from Python. */
int oracle_rx_parse_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n, int zero_trailer,
                          oracle_rx_desc *out) {
    for (uint64_t i = 0; i < n; i++) {
        const int rc = oracle_rx_parse(base + off[i], len[i], off[i], zero_trailer, out + i);
        if (rc != ORACLE_OK) return rc;
    }
    return ORACLE_OK;
}

/* ---------------------------------------------------------------------------------- */
/* Synthetic workloads                                                                 */
/* ---------------------------------------------------------------------------------- */
/* splitmix64 output function (Steele/Lea/Flood 2014) applied to x + golden gamma. */
uint64_t oracle_mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint8_t payload_byte(uint64_t key, uint64_t q) {
    if (key == UINT64_MAX) return (uint8_t)q; /* common.rs:240: e = i as u8 */
    return (uint8_t)(oracle_mix64(key + (q >> 3)) >> (8u * (uint32_t)(q & 7u)));
}

/* Write::handle (queues/send/operations/write.rs:31-96) + send_write_message
 * (common.rs:73-132) + generate_payload_from_msg (net/util.rs:172-186): src 192.168.0.2
 * (common.rs:124), port 4791, ip_id 1, tran_type RC, solicited 0, pkey = msn,
 * RETH len = whole message length on every packet. */
int64_t oracle_synth_write(uint8_t *base, uint64_t stride, uint64_t max_pkts, uint32_t *lens,
                           uint64_t local_va, uint64_t remote_va, uint32_t total_len,
                           uint32_t pmtu, uint32_t rkey, uint32_t dqpn, uint32_t psn0,
                           uint16_t msn, uint32_t dst_ip, uint64_t payload_key) {
    uint32_t nseg = oracle_generate_segments(local_va, total_len, pmtu, NULL, NULL, 0);
    if (nseg > max_pkts) return ORACLE_BUFFER_NOT_LARGE;
    uint64_t *sva = (uint64_t *)malloc(sizeof(uint64_t) * nseg);
    uint32_t *sl = (uint32_t *)malloc(sizeof(uint32_t) * nseg);
    uint8_t *payload = (uint8_t *)malloc(pmtu + 4);
    if (!sva || !sl || !payload) {
        free(sva); free(sl); free(payload);
        return ORACLE_EINVAL;
    }
    oracle_generate_segments(local_va, total_len, pmtu, sva, sl, nseg);
    uint32_t psn = psn0;
    uint64_t rva = remote_va;
    uint64_t msg_off = 0;
    int64_t rc = (int64_t)nseg;
    for (uint32_t i = 0; i < nseg; i++) {
        uint8_t op;
        int ack;
        if (nseg == 1) { op = OP_WRITE_ONLY; ack = 1; }
        else if (i == 0) { op = OP_WRITE_FIRST; ack = 0; }
        else if (i + 1 == nseg) { op = OP_WRITE_LAST; ack = 1; }
        else { op = OP_WRITE_MIDDLE; ack = 0; }
        for (uint32_t q = 0; q < sl[i]; q++) payload[q] = payload_byte(payload_key, msg_off + q);
        oracle_rdma_msg m;
        memset(&m, 0, sizeof m);
        m.kind = 0;
        m.opcode = op;
        m.tran_type = 0;
        m.solicited = 0;
        m.ack_req = (uint8_t)ack;
        m.pkey = msn;
        m.dqpn = dqpn;
        m.psn = psn;
        m.reth_va = rva;
        m.reth_rkey = rkey;
        m.reth_len = total_len;
        m.payload = payload;
        m.payload_len = sl[i];
        uint8_t *pkt = base + (uint64_t)i * stride;
        memset(pkt, 0, stride < 8192 ? stride : 8192); /* util.rs:173: vec![0; 8192] */
        size_t L = 0;
        int w = oracle_packet_write(pkt, stride, &m, 0xC0A80002u, 4791, dst_ip, 4791, 1, &L);
        if (w) { rc = w; break; }
        lens[i] = (uint32_t)L;
        rva += sl[i];
        msg_off += sl[i];
        psn += 1; /* wrapping_add(1), write.rs:64,78 */
    }
    free(sva);
    free(sl);
    free(payload);
    return rc;
}

int64_t oracle_synth_middle_stream(uint8_t *base, uint64_t stride, uint64_t n, uint32_t *lens,
                                   uint64_t remote_va, uint32_t reth_len, uint32_t pmtu,
                                   uint32_t rkey, uint32_t dqpn, uint32_t psn0, uint16_t msn,
                                   uint32_t dst_ip, uint64_t payload_key) {
    uint8_t *payload = (uint8_t *)malloc(pmtu + 4);
    if (!payload) return ORACLE_EINVAL;
    for (uint64_t p = 0; p < n; p++) {
        for (uint32_t q = 0; q < pmtu; q++) payload[q] = payload_byte(payload_key, p * pmtu + q);
        oracle_rdma_msg m;
        memset(&m, 0, sizeof m);
        m.kind = 0;
        m.opcode = OP_WRITE_MIDDLE;
        m.pkey = msn;
        m.dqpn = dqpn;
        m.psn = psn0 + (uint32_t)p;
        m.reth_va = remote_va + p * pmtu;
        m.reth_rkey = rkey;
        m.reth_len = reth_len;
        m.payload = payload;
        m.payload_len = pmtu;
        uint8_t *pkt = base + p * stride;
        memset(pkt, 0, stride);
        size_t L = 0;
        int w = oracle_packet_write(pkt, stride, &m, 0xC0A80002u, 4791, dst_ip, 4791, 1, &L);
        if (w) { free(payload); return w; }
        lens[p] = (uint32_t)L;
    }
    free(payload);
    return (int64_t)n;
}
