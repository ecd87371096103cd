/*
 * include/icrc.h — C-ABI of the MI355X ICRC engine (libicrc_amd.so).
 *
 * The drop-in boundary for the RoCEv2 Invariant-CRC path of Foreverhighness/open-rdma-driver.
 * Every entry point cites the reference interface it replaces (paths relative to the
 * reference root):
 *
 *   compute_icrc(&[u8]) -> u32
 *       blue-rdma-device/src/third_party/net/packet_processor.rs:275-301
 *       (identical copy: rust_driver/src/device/software/packet_processor.rs:275-301,
 *        and rust_driver/src/responser.rs:284-307 `calculate_icrc`)
 *   is_icrc_valid(&mut [u8]) -> Result<bool, PacketProcessorError>
 *       packet_processor.rs:341-353
 *   PacketWriter::{new,src_addr,src_port,dest_addr,dest_port,ip_id,message,write}
 *       packet_processor.rs:150-265 (+ write_ip_udp_header 303-332)
 *
 * Plain pointers and sizes only; no HIP or torch types appear in the signatures (a HIP
 * stream is passed as an opaque `void*`, i.e. a hipStream_t; NULL = the HIP null stream, as in
 * every HIP API; icrc_engine_stream() returns the engine's own non-blocking stream).
 *
 * Conventions
 *   - A packet is a full IPv4 datagram (no Ethernet header) starting at the IPv4 header;
 *     `len` is the IPv4 total length INCLUDING the 4-byte ICRC trailer, whose contents
 *     are ignored by compute.  The ICRC is stored little-endian at [len-4, len).
 *   - Return codes: 0 = OK, negative = error (ICRC_E*).  A CRC mismatch is a result
 *     (ok = 0), never an error.  Nothing aborts; the reference's panics (len < 44) map to
 *     ICRC_EINVAL.
 *   - The caller owns every buffer.  Synchronous calls retain no pointer; *_device calls
 *     borrow their pointers until the stream they were issued on is synchronised.
 *   - All entry points are reentrant.  Scalar calls, and host batches of at most 1024 packets and
 *     8 MiB (one message: configs[0] is 64 x 4156 B), are host messages: the kernel reads the
 *     packets from pinned, device-mapped host memory (the caller's own buffer when the whole span
 *     lies in one pinned allocation and every packet is 4-byte aligned, else a copy in a staging
 *     slot of the calling thread).  By default (ICRC_HOST_RING) a message is a job in the engine's
 *     submission ring: a resident service kernel polls the ring's slots in pinned host memory (the
 *     emulator's doorbell / descriptor-queue model, queues/send/queue.rs:66-100), so a call costs
 *     no kernel launch; the kernel (eight 256-thread workgroups per slot: 32 CUs) ends between jobs after 1 ms
 *     of life or 2 ms without calls and the next call starts it again; a job not done within 2 s
 *     retires the ring (counted in icrc_engine_host_stats out[3]) and the call, and every later
 *     one, runs as a kernel launch instead.  Up to four messages run at once (the emulator's three
 *     threads each get one); more callers wait for a slot.  ICRC_HOST_LAUNCH
 *     (icrc_engine_set_host_path) runs each message as a kernel launch instead, through a
 *     four-stream submitter that merges callers beyond four into one launch.  Larger host batches
 *     serialise per engine on its two pipelined H2D staging buffers; device batches only enqueue on
 *     the caller's stream.  The default-engine registry is lock-protected.
 *   - Every CRC is computed by the HIP kernel on the GPU; there is no CPU fallback.  With
 *     no usable GPU the calls return ICRC_ENODEV.
 */
#ifndef ICRC_AMD_ICRC_H
#define ICRC_AMD_ICRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICRC_OK 0
#define ICRC_EINVAL (-22)  /* bad argument: NULL, len < 44 (reference panics), n too big */
#define ICRC_ENOMEM (-12)  /* host or device allocation failed                           */
#define ICRC_ENODEV (-19)  /* no usable GPU / engine for the requested device             */
#define ICRC_EDEVICE (-5)  /* a HIP runtime call failed                                   */
#define ICRC_ETIMEDOUT (-110) /* a submission ring's kernel did not stop (icrc_engine_destroy, icrc_shutdown) */
/* PacketWriter errors (PacketProcessorError, packet_processor.rs:127-148) */
#define ICRC_EBUFFER_NOT_LARGE (-1000) /* BufferNotLargeEnough(usize)                     */
#define ICRC_ELENGTH_TOO_LONG (-1001)  /* LengthTooLong(usize)                            */
#define ICRC_EINVALID_METADATA (-1002) /* PacketError::InvalidMetadataType                */
#define ICRC_EINVALID_OPCODE (-1003)   /* PacketError::InvalidOpcode                      */

/* Minimum packet: IPv4(20) + UDP(8) + BTH(12) + ICRC(4) (CommonPacketHeader + ICRC_SIZE). */
#define ICRC_MIN_PACKET 44u
/* verify result byte values */
#define ICRC_VERIFY_MISMATCH 0u
#define ICRC_VERIFY_OK 1u
/* device batches: len < 44 (counted in *d_nerr).  Also the short-packet kernel's safety net: a wave
 * whose frame bookkeeping would not terminate (never observed; it exists so that a bug ends in
 * flagged results, not in a hung GPU) reports every packet of its range as BADLEN (compute: ICRC 0)
 * and adds them to *d_nerr — pass d_nerr to see it. */
#define ICRC_VERIFY_BADLEN 0xFFu

typedef struct icrc_engine icrc_engine;

/* ---- ABI version ------------------------------------------------------------------------ */
/* Bumped whenever a struct layout or an entry point's meaning changes.  5: icrc_write_msg is 96 bytes
 * (88 before round 4: imm + a reserved word), the ICRC_WRITE_SEG_BY_REMOTE_VA name is gone (its bit
 * is ICRC_WRITE_RUST_DRIVER, whose meaning grew in round 4), the submission ring. */
#define ICRC_ABI_VERSION 5u
uint32_t icrc_abi_version(void);
/* A binding's start-up check: ICRC_OK when the library implements `abi_version` and the caller's
 * struct sizes are the library's (a Rust #[repr(C)] mirror passes its size_of values), else
 * ICRC_EINVAL — an 88-byte icrc_write_msg stride would misread every message after the first. */
int icrc_abi_check(uint32_t abi_version, size_t write_msg_bytes, size_t rx_desc_bytes, size_t ack_ctx_bytes,
                   size_t synth_desc_bytes);
#define ICRC_ABI_CHECK()                                                                                  \
    icrc_abi_check(ICRC_ABI_VERSION, sizeof(icrc_write_msg), sizeof(icrc_rx_desc), sizeof(icrc_ack_ctx), \
                   sizeof(icrc_synth_desc))

/* ---- engine lifetime ------------------------------------------------------------------ */
/* One engine per GPU: owns the LDS table images in HBM (160 KiB each, plus a 36 KiB compact form the
 * kernels replicate into LDS), a stream and staging. */
int icrc_engine_create(int device, icrc_engine **out);
/* ICRC_EINVAL for a handle that is not a live engine (NULL, destroyed, or gone with icrc_shutdown).
 * ICRC_ETIMEDOUT when the engine's submission ring kernel did not stop within 1 s: the engine is
 * gone, but the ring's stream and memory are left in place (never waited for). */
int icrc_engine_destroy(icrc_engine *engine);
/* Process teardown, before the HIP runtime's own: stops every submission ring, synchronises and
 * destroys every engine (the default ones and those from icrc_engine_create: their handles become
 * invalid) and frees every thread's staging slot.  Afterwards no entry point makes a HIP call: those
 * that need the GPU return ICRC_EDEVICE (engines) / ICRC_ENODEV, icrc_device_count returns 0.  Call
 * it from the host program's exit path (the Python binding registers it with atexit).  Returns
 * ICRC_OK, or ICRC_ETIMEDOUT when a ring kernel did not stop (left in place, as above).  Idempotent. */
int icrc_shutdown(void);
/* Lazily created, lock-protected default engine for `device` (-1 = current HIP device). */
int icrc_engine_default(int device, icrc_engine **out);
int icrc_engine_device_ordinal(const icrc_engine *engine);
/* The engine's own non-blocking stream (a hipStream_t), for callers without one. */
void *icrc_engine_stream(const icrc_engine *engine);
/* Tuning knob for A/B measurement (kernel variants, icrc_kernels.hip launch_mode).  Every value
 * this library accepts gives identical results:
 *   -1   the defaults: uniform strided batches of packets >= 1089 B and batches of at most one
 *        packet per wave (#CUs x 16) take 16; strided batches of shorter packets take 40; larger
 *        ragged batches are split by length in ONE launch (icrc_hybrid_kernel): 40 takes
 *        L <= 1088, the long-packet kernel L >= 1089;
 *   0    one packet per wavefront, not pipelined;
 *   13 / 16 / 17  one packet per wavefront, software-pipelined, one / two CRC chains per wave
 *        (17 = 16 without the raised wave priority around its load bursts);
 *   40   eight packets per wavefront (the oct kernel, packets up to 1088 B; longer ones ride
 *        along on its per-packet path);
 *   140 / 240  the length split as two kernels forked / joined on two streams (240: the
 *        compacting long-packet walker);
 *   301 / 302  the receive parse as one fused pass on any batch (S = 2 / S = 1).
 * Other values: ICRC_EINVAL.  The diagnostics whose results are wrong by design (15, 18, 19,
 * 21-23, 27-30, 33, 41-53, 141-153, 241-253) exist only in the A/B library libicrc_amd_ab.so (built with
 * ICRC_AB_BUILD), which no product path loads. */
int icrc_engine_set_kernel_variant(icrc_engine *engine, int variant);
/* The path of host messages (scalar calls, host batches of at most 1024 packets): */
#define ICRC_HOST_RING 0   /* the submission ring and its resident service kernel (default)         */
#define ICRC_HOST_LAUNCH 1 /* a kernel launch per message (the four-stream submitter)               */
int icrc_engine_set_host_path(icrc_engine *engine, int path);
/* Counters of the engine's submission ring: out[0] jobs run, [1] service-kernel launches, [2] of
 * them relaunches (a call after an idle exit, or a launch that ended under a job), [3] watchdog
 * timeouts.  All zero before the first host message. */
int icrc_engine_host_stats(icrc_engine *engine, uint64_t out[4]);
/* Number of HIP devices visible (0 when no GPU); never fails. */
int icrc_device_count(void);
/* Static library/kernel description (for logs): "icrc_amd <ver> gfx950 ..." */
const char *icrc_version(void);

/* ---- scalar drop-ins (replace compute_icrc / is_icrc_valid) ---------------------------- */
/* compute_icrc, packet_processor.rs:275-301.  Returns the ICRC; *err (may be NULL) gets
 * ICRC_OK or an error code (then the return value is 0).  len in [44, 65535] (an IPv4 packet),
 * else ICRC_EINVAL.  Latency and throughput from 1 and 3 threads: profiles/ (scalar_probe). */
uint32_t icrc_compute(const uint8_t *pkt, size_t len, int *err);
/* is_icrc_valid, packet_processor.rs:341-353.  *ok = 1 when the trailer matches.
 * zero_trailer != 0 reproduces the reference's in-place zeroing of the trailer (350). */
int icrc_verify(uint8_t *pkt, size_t len, int zero_trailer, int *ok);

/* ---- host-resident batches (packets in host memory: descriptor rings, wire buffers) ---- */
/* Packet i is base[off[i] .. off[i]+len[i]).  write_trailer != 0 stores each ICRC LE into
 * its packet's last 4 bytes (what PacketWriter::write does, packet_processor.rs:260-263). */
int icrc_compute_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n,
                       uint32_t *out_icrc, int write_trailer);
/* ok[i] = 1/0 per packet (one byte each).  zero_trailer as icrc_verify. */
int icrc_verify_batch(uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t n,
                      uint8_t *ok, int zero_trailer);
int icrc_compute_batch_ex(icrc_engine *engine, uint8_t *base, const uint64_t *off,
                          const uint32_t *len, uint32_t n, uint32_t *out_icrc, int write_trailer);
int icrc_verify_batch_ex(icrc_engine *engine, uint8_t *base, const uint64_t *off,
                         const uint32_t *len, uint32_t n, uint8_t *ok, int zero_trailer);

/* ---- device-resident batches (all pointers are device pointers; async on `stream`) ----- */
/* d_off/d_len: per-packet (offset, len).  d_out (may be NULL) receives the ICRCs.
 * d_nerr (may be NULL): device uint32 counter incremented once per packet with len < 44
 * (its ICRC is reported as 0 and nothing is written to that packet). */
int icrc_compute_batch_device(icrc_engine *engine, uint8_t *d_base, const uint64_t *d_off,
                              const uint32_t *d_len, uint32_t n, uint32_t *d_out,
                              int write_trailer, uint32_t *d_nerr, void *stream);
int icrc_verify_batch_device(icrc_engine *engine, uint8_t *d_base, const uint64_t *d_off,
                             const uint32_t *d_len, uint32_t n, uint8_t *d_ok, int zero_trailer,
                             uint32_t *d_nerr, void *stream);
/* Uniform batches: packet i at d_base + i*stride, every packet `len` bytes. */
int icrc_compute_strided_device(icrc_engine *engine, uint8_t *d_base, uint64_t stride,
                                uint32_t len, uint32_t n, uint32_t *d_out, int write_trailer,
                                void *stream);
int icrc_verify_strided_device(icrc_engine *engine, uint8_t *d_base, uint64_t stride,
                               uint32_t len, uint32_t n, uint8_t *d_ok, int zero_trailer,
                               void *stream);

/* ---- receive: verify + strip + parse (§8f row 2) ---------------------------------------------
 * For each received IPv4 packet: is_icrc_valid (packet_processor.rs:341-353), then
 * PacketProcessor::to_rdma_message (packet_processor.rs:18-71, packet.rs:286-438) applied to the
 * UDP payload with the ICRC stripped (pkt[28 .. L-4)): the emulator hands the whole datagram,
 * trailer included, to to_rdma_message (device_inner.rs:150) and so reports payloads 4 bytes
 * too long; here payload_len excludes it.  A batch of at most one packet per wave (#CUs x 16)
 * runs as ONE fused kernel; larger ones as two kernels on `stream`: the verify batch, then a
 * descriptor pass that re-reads each packet's first 72 bytes.  With d_ok NULL
 * the two-kernel form keeps the ok bytes in a stream-ordered scratch array (hipMallocAsync /
 * hipFreeAsync on `stream`). */
#define ICRC_RX_OK 0u
#define ICRC_RX_INVALID_OPCODE 1u     /* PacketError::InvalidOpcode (opcode not in 0x06..0x11)   */
#define ICRC_RX_INVALID_TRANS_TYPE 2u /* PacketError::FailedToConvertTransType (tran_type > 6) */
#define ICRC_RX_TRUNCATED 3u          /* L < 44, or headers + pad longer than the packet (the
                                         reference reads out of bounds there)                  */
#define ICRC_RX_SOLICITED 0x01u
#define ICRC_RX_ACK_REQ 0x02u
#define ICRC_RX_HAS_IMM 0x04u
#define ICRC_RX_HAS_SECONDARY_RETH 0x08u
#define ICRC_RX_ACKNOWLEDGE 0x10u /* Metadata::Acknowledge (AETH fields valid), else General */
typedef struct icrc_rx_desc {
    uint64_t reth_va;        /* RETH (General metadata)                                    */
    uint64_t sec_va;         /* secondary RETH (RdmaReadRequest)                            */
    uint64_t payload_offset; /* byte offset of the payload in d_base                        */
    uint32_t payload_len;    /* UDP payload - ICRC - headers - pad (get_packet_real_length) */
    uint32_t reth_rkey, reth_len;
    uint32_t sec_rkey, sec_len;
    uint32_t imm;
    uint32_t dqpn, psn;
    uint32_t aeth_msn;
    uint16_t pkey;
    uint8_t opcode, tran_type;
    uint8_t flags;           /* ICRC_RX_* bits                                               */
    uint8_t pad_cnt;
    uint8_t aeth_code, aeth_value;
    uint8_t icrc_ok;         /* ICRC_VERIFY_OK / _MISMATCH / _BADLEN                          */
    uint8_t status;          /* ICRC_RX_*; on status != OK every parsed field is 0           */
    uint8_t _pad[2];
} icrc_rx_desc; /* 72 bytes */
/* Packet i = d_base[d_off[i] .. + d_len[i]) (d_off / d_len NULL => i * stride / len).  d_ok
 * (may be NULL) receives icrc_ok as in icrc_verify_batch_device; zero_trailer as there. */
int icrc_rx_parse_device(icrc_engine *engine, uint8_t *d_base, const uint64_t *d_off,
                         const uint32_t *d_len, uint64_t stride, uint32_t len, uint32_t n,
                         icrc_rx_desc *d_desc, uint8_t *d_ok, int zero_trailer, uint32_t *d_nerr,
                         void *stream);

/* ---- receive-side auto-ACK (§8a row a5: generate_ack, net/util.rs:134-170) ------------------
 * From the descriptors of icrc_rx_parse_device, the ACK every receive handler sends
 * (write_first.rs:35-82 and the ten other message handlers): needed when the packet parsed
 * (status ICRC_RX_OK), its ICRC verified (icrc_ok == ICRC_VERIFY_OK), it is not an ACK, ack_req
 * is set, its QP is valid (ctx.flags QP_VALID), its memory-region check did not fail (ctx.flags
 * MR_ERROR clear: copy_to_with_key, write_first.rs:35-44 — an abnormal packet is never
 * auto-ACKed) and psn == ctx.expected_psn.  The ACK is generate_ack's
 * 48-byte packet: 192.168.0.3 -> 192.168.0.2, ip_id 1, UDP 4791 -> 4791, BTH {Acknowledge, RC,
 * pkey, dqpn = peer_qpn, psn = expected_psn}, AETH {Ack, 0x1f, msn = pkey} and its ICRC; with
 * ICRC_ACK_UDP_PAYLOAD_ONLY the 20-byte UDP payload generate_ack returns (util.rs:167-169).
 * Slot i is d_out + i * out_stride (out_stride % 4 == 0, d_out 4-byte aligned); d_out_len[i] =
 * 48 / 20, or 0 when no ACK is due (its slot is not written). */
typedef struct icrc_ack_ctx {
    uint32_t peer_qpn;     /* qp_context.peer_qpn() of the packet's QP (dqpn)                */
    uint32_t expected_psn; /* qp_context.expected_psn() before this packet                    */
    uint32_t flags;        /* ICRC_ACK_CTX_* below                                            */
} icrc_ack_ctx;
#define ICRC_ACK_CTX_QP_VALID 0x1u /* the QP exists and is not in the error state (qp_error,
                                      is_error(): write_first.rs:39-60)                          */
#define ICRC_ACK_CTX_MR_ERROR 0x2u /* the packet's MR / key check failed (mr_error = copy_to_with_key
                                      (msg).is_err(), write_first.rs:35): no ACK                 */
#define ICRC_ACK_UDP_PAYLOAD_ONLY 0x1u
int icrc_ack_from_rx_device(icrc_engine *engine, const icrc_rx_desc *d_desc, const icrc_ack_ctx *d_ctx, uint32_t n,
                            uint8_t *d_out, uint32_t out_stride, uint32_t *d_out_len, uint32_t flags,
                            void *stream);

/* ---- batched IPv4 header checksum (§8f row 4) ----------------------------------------------
 * calculate_ipv4_checksum (rust_driver/src/responser.rs:321-338): the one's-complement sum of
 * the ten big-endian 16-bit words of the 20-byte IPv4 header at d_base + off (d_off NULL =>
 * i * stride), complemented.  fill == 0: over the header as stored (a header carrying a valid
 * checksum gives 0); fill != 0: with bytes 10-11 taken as 0 and the result then stored there
 * big-endian (responser.rs:198-201).  d_csum (may be NULL) receives the u16 per packet.  The
 * ICRC masks bytes 10-11, so filling never changes a packet's ICRC. */
int icrc_ipv4_checksum_device(icrc_engine *engine, uint8_t *d_base, const uint64_t *d_off,
                              uint64_t stride, uint32_t n, uint16_t *d_csum, int fill, void *stream);

/* ---- packet synthesis on the device (bench inputs; precursor of the fused packetizer) --- */
/* Packet i = header template d_hdr[hdr_index*64 .. +hdr_len) ‖ payload ‖ zero pad ‖ zero
 * ICRC slot, written at d_base + offset.  Payload byte q = byte ((pos+q) & 7) of
 * splitmix64_mix(payload_key + ((pos+q) >> 3)) — the same function as the oracle's
 * oracle_mix64 — so that host and device synthesise identical bytes. */
typedef struct icrc_synth_desc {
    uint64_t offset;
    uint64_t payload_key;
    uint64_t payload_pos;
    uint32_t hdr_len;     /* <= 64, multiple of 4 */
    uint32_t payload_len; /* bytes before pad */
    uint32_t total_len;   /* L (IPv4 total length incl. ICRC) */
    uint32_t hdr_index;
} icrc_synth_desc;
int icrc_synth_device(icrc_engine *engine, uint8_t *d_base, const icrc_synth_desc *d_desc,
                      const uint8_t *d_hdr, uint32_t n, void *stream);

/* ---- fused send packetizer (§8f rows 1 + 3) -------------------------------------------------
 * The emulator's whole send step for RDMA WRITE / READ RESPONSE messages, on the device, in one
 * kernel: MTU segmentation (generate_segments_from_request, queues/send/operations/
 * common.rs:152-176), per-packet opcode / PSN / ack_req / RETH (write.rs:31-96,
 * read_response.rs:30-95, send_write_message common.rs:73-132), header serialisation and
 * payload copy (PacketWriter::write, packet_processor.rs:210-265), zero pad, and the ICRC
 * (computed from the words in registers, no re-read) written as the trailer.
 *
 * Packet s of message m is written at d_wire + m.out_offset + s * m.slot_stride; its length
 * goes to d_pkt_len[m.first_packet + s] and its ICRC to d_icrc[m.first_packet + s] (both may
 * be NULL).  Payload bytes come from d_src[m.payload_offset + segment start ...].  The
 * fast path needs (payload_offset - seg_va) % 4 == 0, where seg_va is the segmentation VA
 * (local_va; remote_va under ICRC_WRITE_RUST_DRIVER), and out_offset, slot_stride % 4 == 0;
 * other messages take a byte-wise path with identical results.  A packet longer than 65535 bytes
 * (IPv4 total length; PacketWriter::write returns LengthTooLong, packet_processor.rs:226-227) is
 * not written and reports length 0, like one that does not fit. */
typedef struct icrc_write_msg {
    uint64_t local_va;       /* source VA of the payload: drives the first segment length; read
                                requests: the secondary RETH va (the local SGE, read.rs:69-73) */
    uint64_t remote_va;      /* RETH va of the first packet */
    uint64_t payload_offset; /* byte offset of the message payload in d_src */
    uint64_t out_offset;     /* byte offset of packet 0 in d_wire */
    uint32_t total_len;      /* sge.len: bytes to send, drives segmentation (read requests: the
                                secondary RETH len; ICRC_WRITE_RUST_DRIVER: the SG list's total
                                length, sg_list.get_total_length(), logic.rs:207) */
    uint32_t reth_len;       /* common.total_len: the RETH len of every packet (common.rs:113);
                                ICRC_WRITE_RUST_DRIVER: only FIRST packets carry it (logic.rs:121-125,
                                224-228), the others their own lengths (240, 265) */
    uint32_t pmtu;           /* 256 .. 4096 (WRITE / READ RESPONSE) */
    uint32_t rkey;
    uint32_t dqpn;
    uint32_t psn;            /* PSN of packet 0 (wraps at 24 bits) */
    uint32_t src_ip, dst_ip; /* host order; the emulator uses 192.168.0.2 (common.rs:124) */
    uint32_t first_packet;   /* index of packet 0 in the flattened packet arrays */
    uint32_t npackets;       /* icrc_write_segment_count(local_va, total_len, pmtu); 1 for a read request */
    uint32_t slot_stride;    /* bytes between consecutive packets of this message */
    uint16_t msn;            /* carried in the BTH pkey field (common.rs:91-92) */
    uint16_t ip_id;          /* generate_payload_from_msg uses 1 (net/util.rs:179) */
    uint8_t kind;            /* ICRC_MSG_* below */
    uint8_t tran_type;       /* RC = 0 */
    uint8_t flags;           /* ICRC_WRITE_* below */
    uint8_t _pad;
    uint32_t lkey;           /* read requests: the secondary RETH rkey (sge.local_key) */
    uint32_t imm;            /* ImmDt of a WRITE_WITH_IMM descriptor (ICRC_WRITE_WITH_IMM) */
    uint32_t _rsvd;          /* 0 */
} icrc_write_msg; /* 96 bytes */
#define ICRC_MSG_WRITE 0u         /* Write::handle (write.rs:31-96): WRITE FIRST/MIDDLE/LAST/ONLY  */
#define ICRC_MSG_READ_RESPONSE 1u /* ReadResponse::handle (read_response.rs:30-95)                 */
#define ICRC_MSG_READ_REQUEST 2u  /* Read::handle (read.rs:33-89): one 76-byte packet, opcode 0x0C,
                                     RETH {remote_va, rkey, reth_len} + secondary RETH {local_va,
                                     lkey, total_len}, no payload                                 */
/* Fill the IPv4 header checksum (RFC 791, as smoltcp's fill_checksum does when the emulator
 * builds the frame, net_agent.rs:93; calculate_ipv4_checksum, responser.rs:321-338).  The
 * ICRC masks those bytes, so it is the same either way.  Default: 0, as PacketWriter leaves it. */
#define ICRC_WRITE_FILL_IPV4_CSUM 0x01u
/* The rust_driver software device's send rule, BlueRDMALogic::send (rust_driver/src/device/software/
 * logic.rs:109-134, 168-271) instead of the emulator's (write.rs:31-96):
 *   - segmentation on the REMOTE VA: first packet = pmtu - remote_va % pmtu (get_first_packet_max_length,
 *     rust_driver/src/utils.rs:19-25); npackets = calculate_packet_cnt (utils.rs:28-33), which
 *     icrc_write_segment_count(remote_va, total_len, pmtu) returns;
 *   - opcodes from the descriptor's is_first / is_last (ToCardWriteDescriptor, types.rs:557-609): a
 *     continuation descriptor (ICRC_WRITE_NOT_FIRST) starts with MIDDLE, one that is not the message's
 *     end (ICRC_WRITE_NOT_LAST) ends with MIDDLE; a one-packet descriptor takes ONLY / FIRST / LAST
 *     (write_only_opcode_with_imm: neither flag set -> ONLY, NOT_LAST -> FIRST, otherwise LAST);
 *   - RETH len: reth_len (common.total_len) on a FIRST packet, the packet's own payload length on a
 *     one-packet or first continuation packet (:121-125, :224-228), pmtu on MIDDLE (:240), the remaining
 *     length on the last packet (:265); RETH va = remote_va + bytes before the packet (:229, 244, 264);
 *   - ICRC_WRITE_WITH_IMM (kind WRITE): LAST / ONLY become WRITE_LAST / WRITE_ONLY_WITH_IMMEDIATE (0x09 /
 *     0x0B) carrying ImmDt = imm after the RETH (RdmaHeaderReqBthRethImm, packet.rs:354-390);
 *   - ack_req and solicited are clear on every packet (RdmaMessageMetaCommon, logic.rs:175-186);
 *     ICRC_WRITE_ACK_REQ / _SOLICITED still set them when given.
 * PSN +1 per packet (24-bit wrap, Psn::wrapping_add, types.rs:180-183), as in both variants. */
#define ICRC_WRITE_RUST_DRIVER 0x02u
/* (Until round 3 this bit was named ICRC_WRITE_SEG_BY_REMOTE_VA and switched only the segmentation
 * VA.  The name is gone so that such callers fail to compile instead of silently getting the whole
 * rust_driver rule; ICRC_ABI_VERSION 5.) */
/* RdmaMessageMetaCommon::solicited on every packet of the message (BTH byte 1 bit 7, packet.rs:
 * 104-110); the emulator's own send paths leave it false (common.rs:90, read.rs:47). */
#define ICRC_WRITE_SOLICITED 0x04u
/* Read requests: ack_req (the request is IbvSendSignaled, read.rs:37).  WRITE / READ RESPONSE
 * packets carry ack_req on their LAST / ONLY packet regardless (write.rs:41-90). */
#define ICRC_WRITE_ACK_REQ 0x08u
/* Emit the UDP payload only (BTH .. ICRC, L - 28 bytes) at each slot: the form
 * generate_payload_from_msg returns and NetAgent::send_to takes (net/util.rs:183-185).  The ICRC
 * is the same (it covers the masked IPv4 / UDP header, which is not stored); d_pkt_len reports
 * L - 28, the bytes written. */
#define ICRC_WRITE_UDP_PAYLOAD_ONLY 0x10u
/* ICRC_WRITE_RUST_DRIVER descriptor flags (ToCardWriteDescriptor, types.rs:548-555; ignored otherwise):
 * is_first = false, is_last = false, and a WriteWithImm descriptor's imm (types.rs:641-648). */
#define ICRC_WRITE_NOT_FIRST 0x20u
#define ICRC_WRITE_NOT_LAST 0x40u
#define ICRC_WRITE_WITH_IMM 0x80u
/* Number of packets generate_segments_from_request yields (common.rs:152-176) for a message
 * whose segmentation VA is `va` (local_va, or remote_va under ICRC_WRITE_RUST_DRIVER);
 * 0 if pmtu == 0. */
uint32_t icrc_write_segment_count(uint64_t local_va, uint32_t total_len, uint32_t pmtu);
/* Wire length of segment s (IPv4 + UDP + BTH + RETH + payload + pad + ICRC). */
uint32_t icrc_write_packet_len(uint64_t local_va, uint32_t total_len, uint32_t pmtu, uint32_t s);
/* d_msgs is device memory, sorted by first_packet, first_packet[0] == 0, packets contiguous
 * (first_packet[m+1] == first_packet[m] + npackets[m]), sum of npackets == npackets.  A packet
 * whose slot would run past wire_bytes (or whose payload lies outside d_src) is not written:
 * its d_pkt_len entry is 0. */
int icrc_write_packetize_device(icrc_engine *engine, const uint8_t *d_src, uint64_t src_bytes,
                                const icrc_write_msg *d_msgs, uint32_t nmsgs, uint32_t npackets,
                                uint8_t *d_wire, uint64_t wire_bytes, uint32_t *d_pkt_len,
                                uint32_t *d_icrc, void *stream);

/* ---- packet writer (PacketWriter, packet_processor.rs:150-265) -------------------------- */
/* Flattened RdmaMessage (third_party/net/types.rs; Metadata::General / ::Acknowledge). */
typedef struct icrc_rdma_msg {
    uint8_t kind;   /* 0 = Metadata::General, 1 = Metadata::Acknowledge */
    uint8_t opcode; /* ToHostWorkRbDescOpcode (third_party/queues.rs:393-425) */
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
    const uint8_t *payload; /* one scatter-gather element (PayloadInfo) */
    uint64_t payload_len;
} icrc_rdma_msg;

/* Header bytes only (IPv4/UDP/BTH/ext) into buf[0 .. 28+hdr); no payload, no ICRC.
 * *out_hdr_len = 28 + header length; *out_total_len = L.  Used to build synth templates. */
int icrc_packet_headers(uint8_t *buf, size_t buf_len, const icrc_rdma_msg *msg, uint32_t src_ip,
                        uint16_t src_port, uint32_t dst_ip, uint16_t dst_port, uint16_t ip_id,
                        size_t *out_hdr_len, size_t *out_total_len);
/* PacketWriter::write: headers + payload + ICRC (ICRC on the GPU).  *out_len = L. */
int icrc_packet_write(uint8_t *buf, size_t buf_len, const icrc_rdma_msg *msg, uint32_t src_ip,
                      uint16_t src_port, uint32_t dst_ip, uint16_t dst_port, uint16_t ip_id,
                      size_t *out_len);
/* write_ip_udp_header, packet_processor.rs:307-332 (addresses in host order a<<24|..|d). */
void icrc_write_ip_udp_header(uint8_t *buf, uint32_t src_ip, uint16_t src_port, uint32_t dst_ip,
                              uint16_t dst_port, uint16_t total_length, uint16_t ip_id);
/* Header composite length (BTH + extension headers) for an opcode (packet.rs:427-438), or
 * ICRC_EINVALID_OPCODE. */
int icrc_rdma_header_len(uint8_t opcode);

/* ---- host-only helpers (no GPU needed) -------------------------------------------------- */
/* The 160 KiB LDS table image the kernels build in LDS (layout documented in DESIGN.md).  With
 * nwords >= 40960 + 9216 the buffer also receives the compact form the engine keeps after the
 * image in HBM and the kernels replicate into LDS: the 1024 distinct bulk entries, then the final
 * tables. */
int icrc_table_image(uint32_t *out_words, uint32_t nwords);
/* The oct kernel's image (eight packets per wavefront): M^8 bulk, M^(8 - (l & 7)) final. */
int icrc_table_image_oct(uint32_t *out_words, uint32_t nwords);
/* Removed in ABI 5 with the quad kernels; still exported (one release) so that old dynamic links
 * resolve.  Always returns ICRC_EINVAL. */
int icrc_table_image_quad(uint32_t *out_words, uint32_t nwords);

#ifdef __cplusplus
}
#endif
#endif /* ICRC_AMD_ICRC_H */
