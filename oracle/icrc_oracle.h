/*
 * oracle/icrc_oracle.h — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the reference's ICRC path (Foreverhighness/open-rdma-driver,
 * blue-rdma-device/src/third_party/net/{packet_processor,packet,types}.rs and the emulator
 * callers in net/util.rs + queues/send/operations/{common,write}.rs).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 *
 * Parity pinning: the restatement is checked against the reference's own known-answer
 * vectors (packet_processor.rs:367-388, responser.rs:348-393, net/util.rs:225-239) and
 * against Python zlib.crc32 fixtures committed under tests/golden/.
 *
 * The CRC arithmetic lives in the third-party crate crc32fast 1.4.2 (Cargo.lock:230-236),
 * which is not vendored in /root/reference; its published algorithm is CRC-32/ISO-HDLC
 * (reflected poly 0xEDB88320, init 0xFFFFFFFF, xorout 0xFFFFFFFF), restated here.
 */
#ifndef ICRC_ORACLE_H
#define ICRC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes (mirror PacketProcessorError, packet_processor.rs:127-148). */
#define ORACLE_OK 0
#define ORACLE_EINVAL (-22)            /* reference panics (short buffer)           */
#define ORACLE_BUFFER_NOT_LARGE (-1000) /* BufferNotLargeEnough(usize)              */
#define ORACLE_LENGTH_TOO_LONG (-1001)  /* LengthTooLong(usize)                     */
#define ORACLE_INVALID_METADATA (-1002) /* PacketError::InvalidMetadataType          */
#define ORACLE_INVALID_OPCODE (-1003)   /* PacketError::InvalidOpcode                */

/* Opcodes: ToHostWorkRbDescOpcode (third_party/queues.rs:393-425). */
enum {
    OP_WRITE_FIRST = 0x06,
    OP_WRITE_MIDDLE = 0x07,
    OP_WRITE_LAST = 0x08,
    OP_WRITE_LAST_IMM = 0x09,
    OP_WRITE_ONLY = 0x0a,
    OP_WRITE_ONLY_IMM = 0x0b,
    OP_READ_REQUEST = 0x0c,
    OP_READ_RESP_FIRST = 0x0d,
    OP_READ_RESP_MIDDLE = 0x0e,
    OP_READ_RESP_LAST = 0x0f,
    OP_READ_RESP_ONLY = 0x10,
    OP_ACK = 0x11,
};

/* A flattened RdmaMessage (types.rs RdmaMessage / Metadata / PayloadInfo). */
typedef struct oracle_rdma_msg {
    uint8_t kind; /* 0 = Metadata::General, 1 = Metadata::Acknowledge */
    uint8_t opcode;
    uint8_t tran_type; /* ToHostWorkRbDescTransType, RC = 0 */
    uint8_t solicited;
    uint8_t ack_req;
    uint8_t aeth_code;
    uint8_t aeth_value;
    uint8_t has_imm;
    uint8_t has_secondary_reth;
    uint8_t _pad0[3];
    uint16_t pkey;
    uint16_t _pad1;
    uint32_t dqpn;
    uint32_t psn;
    uint32_t msn;
    uint32_t imm;
    uint64_t reth_va;
    uint32_t reth_rkey;
    uint32_t reth_len;
    uint64_t sec_va;
    uint32_t sec_rkey;
    uint32_t sec_len;
    const uint8_t *payload; /* one SG element */
    uint64_t payload_len;
} oracle_rdma_msg;

/* --- CRC core (crc32fast::Hasher semantics: zlib-style chaining) --------------------- */
uint32_t oracle_crc32(uint32_t crc, const uint8_t *p, size_t n);

/* --- ICRC (packet_processor.rs:268-353) --------------------------------------------- */
int oracle_compute_icrc(const uint8_t *pkt, size_t len, uint32_t *out);
int oracle_is_icrc_valid(uint8_t *pkt, size_t len, int *ok);
/* Batch helpers used by tests / cpu_baseline: (offset,len) arrays. */
int oracle_compute_icrc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                              uint64_t n, uint32_t *out);

/* --- Packet synthesis (packet_processor.rs:150-265,303-332; packet.rs:100-243) ------- */
void oracle_write_ip_udp_header(uint8_t *buf, uint32_t src_ip, uint16_t src_port, uint32_t dst_ip,
                                uint16_t dst_port, uint16_t total_length, uint16_t ip_id);
int oracle_header_len(uint8_t opcode);
int oracle_packet_write(uint8_t *buf, size_t buf_len, const oracle_rdma_msg *msg, uint32_t src_ip,
                        uint16_t src_port, uint32_t dst_ip, uint16_t dst_port, uint16_t ip_id,
                        size_t *out_len);
uint32_t oracle_pad_cnt(uint64_t payload_len);

/* net/util.rs:134-170: returns the 20-byte UDP payload of the 48-byte ACK packet. */
int oracle_generate_ack(uint16_t pkey, uint32_t peer_qpn, uint32_t expected_psn, uint8_t *pkt48,
                        uint8_t *udp_payload20);

/* common.rs:152-176 */
uint32_t oracle_generate_segments(uint64_t va, uint32_t len, uint32_t path_mtu, uint64_t *seg_va,
                                  uint32_t *seg_len, uint32_t max_segs);

/* rust_driver's send rule, BlueRDMALogic::send (rust_driver/src/device/software/logic.rs:109-134,
 * 168-271) for a WRITE / WRITE_WITH_IMM / READ_RESP descriptor (ToCardWriteDescriptor,
 * types.rs:548-617).  One entry per RdmaMessage handed to NetSendAgent::send, in order; the payload
 * is bytes [payload_off, payload_off + payload_len) of the descriptor's SG list (SGList::cut). */
typedef struct oracle_write_desc {
    uint64_t raddr;     /* common.raddr */
    uint32_t total_len; /* common.total_len */
    uint32_t sge_len;   /* sg_list.get_total_length() */
    uint32_t pmtu;      /* u32::from(&common.pmtu) */
    uint32_t psn;       /* common.psn */
    uint32_t imm;       /* WriteWithImm's imm */
    uint8_t is_resp;    /* ToCardWorkRbDescOpcode::ReadResp */
    uint8_t is_first, is_last, has_imm;
} oracle_write_desc;
typedef struct oracle_logic_pkt {
    uint64_t reth_va;
    uint32_t psn, reth_len, imm, payload_off, payload_len;
    uint8_t opcode, has_imm, _pad[2];
} oracle_logic_pkt;
/* Returns the number of messages (fills at most max_out). */
uint32_t oracle_logic_send(const oracle_write_desc *d, oracle_logic_pkt *out, uint32_t max_out);

/* responser.rs:321-338 (IPv4 header checksum, §8f row 4). */
uint16_t oracle_ipv4_checksum(const uint8_t *hdr20);

/* --- Receive: is_icrc_valid + to_rdma_message on the stripped UDP payload (§8f row 2) --- */
/* Same field layout as the product's icrc_rx_desc (include/icrc.h), declared independently. */
typedef struct oracle_rx_desc {
    uint64_t reth_va, sec_va, payload_offset;
    uint32_t payload_len, reth_rkey, reth_len, sec_rkey, sec_len, imm, dqpn, psn, aeth_msn;
    uint16_t pkey;
    uint8_t opcode, tran_type, flags, pad_cnt, aeth_code, aeth_value, icrc_ok, status;
    uint8_t _pad[2];
} oracle_rx_desc;
/* pkt = the IPv4 packet at byte offset `off` of the caller's buffer; zero_trailer as
 * is_icrc_valid.  Fills *d; returns 0. */
int oracle_rx_parse(uint8_t *pkt, uint32_t len, uint64_t off, int zero_trailer, oracle_rx_desc *d);
int oracle_rx_parse_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n, int zero_trailer,
                          oracle_rx_desc *out);

/* --- Synthetic workloads ----------------------------------------------- */
uint64_t oracle_mix64(uint64_t x);
/* Emulator WRITE send path (write.rs:31-96 + common.rs:73-132 + util.rs:172-186):
 * one RDMA WRITE of `total_len` bytes from local `local_va` to `remote_va`, segmented at
 * `pmtu`; every packet written (full IPv4 packet incl. ICRC) at base + i*stride.
 * payload byte q of the message = byte (q & 7) of oracle_mix64(payload_key + (q >> 3))
 * (payload_key == UINT64_MAX: the `i as u8` pattern of common.rs:240).
 * Returns the number of packets, fills lens[] (L per packet). */
int64_t oracle_synth_write(uint8_t *base, uint64_t stride, uint64_t max_pkts, uint32_t *lens,
                           uint64_t local_va, uint64_t remote_va, uint32_t total_len,
                           uint32_t pmtu, uint32_t rkey, uint32_t dqpn, uint32_t psn0,
                           uint16_t msn, uint32_t dst_ip, uint64_t payload_key);

/* A stream of `n` WRITE_MIDDLE packets of one QP: packet p carries
 * message bytes [p*pmtu, (p+1)*pmtu), psn = psn0 + p, RETH va = remote_va + p*pmtu,
 * RETH len = reth_len; other fields as oracle_synth_write. */
int64_t oracle_synth_middle_stream(uint8_t *base, uint64_t stride, uint64_t n, uint32_t *lens,
                                   uint64_t remote_va, uint32_t reth_len, uint32_t pmtu,
                                   uint32_t rkey, uint32_t dqpn, uint32_t psn0, uint16_t msn,
                                   uint32_t dst_ip, uint64_t payload_key);

/* --- CPU baseline (icrc_fast.c): crc32fast-equivalent PCLMULQDQ folding core ---------- */
uint32_t fast_crc32_slice16(uint32_t crc, const uint8_t *p, size_t n);
uint32_t fast_crc32(uint32_t crc, const uint8_t *p, size_t n); /* pclmul when >= 128 B */
int fast_compute_icrc(const uint8_t *pkt, size_t len, uint32_t *out);
/* Time-bounded batch: ICRC of packets base + i*stride (len each) for i in [0,n), using
 * `threads` POSIX threads; returns elapsed seconds, writes out[]. */
double fast_icrc_strided_timed(const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n,
                               uint32_t *out, int threads);
/* The emulator send-path cost model (util.rs:172-186): per packet an 8 KiB vec![0; 8192]
 * + payload copy in + ICRC + UDP-payload copy out (to_vec). Returns elapsed seconds. */
double fast_emulator_path_timed(const uint8_t *base, uint64_t stride, uint32_t len, uint64_t n,
                                uint32_t *out);
/* is_icrc_valid (packet_processor.rs:341-353) with the crc32fast-equivalent core over packets
 * base + i*stride, `threads` POSIX threads: ok[i] = 1/0; zero != 0 zeroes each trailer in place
 * (line 350) — then the buffer holds zero trailers afterwards.  Returns elapsed seconds. */
double fast_verify_strided_timed(uint8_t *base, uint64_t stride, uint32_t len, uint64_t n, uint8_t *ok,
                                 int threads, int zero);
/* configs[0]: the emulator's compute + verify round trip for packets (off[i], len[i]) of `base`
 * (one QP's WRITE message), `reps` times per thread on `threads` threads, each thread on its own
 * copy of the message.  Per packet: the send path of fast_emulator_path_timed (vec![0; 8192],
 * payload copy in, compute_icrc, trailer store, UDP-payload copy out), then the receive check on
 * the received bytes (is_icrc_valid with the in-place trailer zeroing).  *bad = packets whose
 * verify failed (0 expected).  Returns elapsed seconds. */
double fast_c0_roundtrip_timed(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                               int threads, int reps, uint64_t *bad);

#ifdef __cplusplus
}
#endif
#endif
