/*
 * otc.h -- public C API of the MI355X (gfx950) bulk symmetric-cipher engine.
 *
 * Layers (re-designed MI355X-first):
 *   L1/L2 device kernels  -> otc_aes_* / otc_rc4_* / otc_xor  (device pointers,
 *                            asynchronous on a caller-supplied hipStream_t)
 *   L3 engine runtime     -> otc_ctx_* (persistent per-device state, tables,
 *                            streams, pinned staging ring) and otc_stream_*
 *                            (host-memory pipelined H2D | kernel | D2H)
 *   L4 multi-GPU          -> otc_multi_* (single-process RCCL over xGMI) ; the
 *                            one-process-per-GPU path lives in
 *                            our_tree_amd/parallel (torch.distributed / RCCL)
 *
 * Reference counterparts: BlockCipher/AES host class
 * (/root/reference/aes-gpu/Source/BlockCipher.h:48-107, AES.h:84-147,
 * AES.cu:50-282) and the CUDA kernels (AES.cu:284-502).  Unlike the reference,
 * every entry point returns an error code (no silent launch failures,
 * AES.cu:250), nothing is allocated per call, and any length is accepted.
 *
 * Streams are passed as `void *` (a hipStream_t; NULL = default stream) so the
 * header is usable from plain C and from ctypes.
 */
#ifndef OTC_H
#define OTC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- errors -------------------------------------------------------------- */
#define OTC_OK 0
#define OTC_ERR_ARG -1        /* bad argument (length, key size, alignment) */
#define OTC_ERR_HIP -2        /* a HIP runtime call failed; see otc_last_error() */
#define OTC_ERR_RCCL -3       /* an RCCL call failed */
#define OTC_ERR_UNSUPPORTED -4
#define OTC_ERR_NOMEM -5

const char *otc_last_error(void);

/* ---- keys ---------------------------------------------------------------- */
#define OTC_DIR_ENCRYPT 1
#define OTC_DIR_DECRYPT 0

/* Expanded key passed BY VALUE as a kernel argument, so round keys land in
 * SGPRs (wave-uniform) with no per-launch copy.  rk: LE column words as in
 * aes_export_rk32(); for OTC_DIR_DECRYPT the equivalent-inverse schedule. */
typedef struct {
    uint32_t rk[60];
    int32_t nr;   /* 10 / 12 / 14 */
    int32_t dir;  /* OTC_DIR_* */
    int32_t bits; /* 128 / 192 / 256 */
    int32_t pad;
} otc_aes_key;

int otc_aes_key_init(otc_aes_key *k, const uint8_t *key, int bits, int dir);

/* ---- implementation selection ------------------------------------------- */
#define OTC_IMPL_AUTO 0     /* the measured winner (docs/PERF.md rounds 5-6): bitsliced for CTR calls >= 2 GiB
                               (AES-256: >= 1 GiB), the persistent T-table CTR kernel from 512 MiB; for ECB / CBC / CFB decryption and the power-of-two segment
                               decryptions the split below from 2 GiB and the persistent T-table claim kernel
                               alone from 512 MiB; segment encryption: the persistent T-table claim kernel from
                               1 GiB; the grid T-table otherwise
                               (OTC_IMPL=ttable|bitslice|split env overrides for the whole process, each where it
                               applies: split for ECB and the decryptions only) */
#define OTC_IMPL_TTABLE 1   /* LDS-resident replicated T-table kernel */
#define OTC_IMPL_BITSLICE 2 /* bitsliced VALU kernel alone: 32 blocks per lane (CTR, ECB, the decryptions; their
                               claim kernels take every 2048-block unit and one T-table workgroup the blocks past
                               the last); segment encryption has no VALU kernel and runs the T-table */
#define OTC_IMPL_SPLIT 3    /* the T-table and the bitsliced kernel CONCURRENTLY over one buffer, each on a
                               pooled CU-masked stream, co-resident on every CU -- LDS and VALU busy at once --
                               claiming units from one counter: ECB, the CBC / CFB decryptions and the segment
                               decryptions ("auto" for these >= 2 GiB).  CTR has no split (it lost to the
                               bitsliced kernel on both HIP runtimes, removed in round 6): a CTR call with
                               OTC_IMPL_SPLIT takes the auto choice */

/* The kernel family `impl` resolves to for a call of nbytes with a bits-bit
 * key (mode 1: CTR, 0: ECB encryption, 2: ECB / CBC decryption, 3: CFB128
 * decryption, 4: CBC / CFB128 decryption of power-of-two segments, 5: CBC /
 * CFB128 encryption of segments < 8 MiB); -1 for an invalid impl or mode. */
int otc_pick_impl(int impl, int bits, int mode, uint64_t nbytes);
/* What the calling thread's last AES call ran: OTC_IMPL_TTABLE,
 * OTC_IMPL_BITSLICE or OTC_IMPL_SPLIT (OTC_IMPL_AUTO before any call).  Set
 * by otc_aes_ctr / _rfc3686 / _ctr_stream, otc_aes_ecb, the CBC / CFB128
 * decryptions and every segment call; a split or bitsliced request that fell
 * back to the T-table (too few units, no memory for the claim counter) reports
 * OTC_IMPL_TTABLE. */
int otc_last_impl(void);
/* Split accounting, a profiling mode (off by default): with
 * otc_split_stats(1) every split call on this thread waits for its kernels
 * and records its claim counter; otc_split_last_units then gives the units
 * the bitsliced side (front) and the T-table side (back) took in the last
 * such call, of nunits (2048-block units, or 64-segment units for segment
 * encryption).  Under impl "bitslice" front == nunits. */
void otc_split_stats(int on);
/* Why the calling thread's last split / bitsliced-claim request ran the
 * T-table alone ("" when it did not fall back): too few claim units, no
 * memory for the claim counter, the per-device pool of auxiliary streams
 * exhausted (at most 4 concurrent split calls per device, each holding two
 * dedicated hardware queues), or the bitsliced half failing to launch. */
const char *otc_split_fallback_reason(void);
int otc_split_last_units(uint64_t *front, uint64_t *back, uint64_t *nunits);
/* Diagnostic builds only (-DOTC_SPLIT_TRACE=1): copy out and reset the
 * wave-start records of the split's kernels (which: 0 T-table, 1 bitsliced),
 * pairs {s_memrealtime, tag << 32 | HW_ID}; returns the count, or -1
 * in the shipped build. */
int otc_split_trace(int which, unsigned long long *buf, int max);

/* ---- device ops (device pointers; async on `stream`) ---------------------
 * All functions accept any byte length; the trailing partial block of CTR is
 * handled inside the kernel.  ECB/CBC lengths must be multiples of 16.
 * In-place (in == out) is allowed except for otc_aes_cbc_decrypt and
 * otc_aes_cfb128_decrypt (they read the previous ciphertext block).
 */
int otc_aes_ecb(const void *in, void *out, size_t nbytes, const otc_aes_key *k, int impl,
                void *stream);

/* CTR with a full 128-bit big-endian counter starting at ctr0 (the semantics
 * of aes_crypt_ctr with nc_off == 0).  `block_offset` is added to ctr0 first
 * (128-bit add with carry) -- this is how shards of one stream are encrypted
 * independently. */
int otc_aes_ctr(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                const uint8_t ctr0[16], uint64_t block_offset, int impl, void *stream);

/* Resumable CTR stream on device buffers with the PolarSSL context semantics
 * (reference aes-modes/aes.c:869-900): nonce_counter = counter of the NEXT
 * block to generate, stream_block = keystream of the current block, nc_off =
 * bytes of it already used.  Calls may split the stream at any byte; in and
 * out may be misaligned but must share their alignment modulo 16.  The
 * context is updated on return (the launches are asynchronous on `stream`). */
typedef struct {
    uint8_t nonce_counter[16];
    uint8_t stream_block[16];
    size_t nc_off;
} otc_aes_ctr_ctx;
int otc_aes_ctr_ctx_init(otc_aes_ctr_ctx *ctx, const uint8_t nonce_counter[16]);
int otc_aes_ctr_stream(otc_aes_ctr_ctx *ctx, const otc_aes_key *k, size_t length, const void *in, void *out,
                       int impl, void *stream);

/* CTR with the AES-NI/RFC 3686 counter layout nonce[4] || ivec[8] || BE32(1),
 * the low 8 bytes incremented as a 64-bit big-endian integer
 * (reference aesni.c:120-152). */
int otc_aes_ctr_rfc3686(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                        const uint8_t nonce[4], const uint8_t ivec[8], uint64_t block_offset,
                        int impl, void *stream);

/* CBC decryption (parallel): P_i = D(C_i) ^ C_{i-1}, C_{-1} = iv.  _impl:
 * with a kernel choice (OTC_IMPL_*; the plain form is OTC_IMPL_AUTO). */
int otc_aes_cbc_decrypt(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                        const uint8_t iv[16], void *stream);
int otc_aes_cbc_decrypt_impl(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                             const uint8_t iv[16], int impl, void *stream);

/* CBC encryption over `nseg` independent segments of `seg_bytes` each
 * (contiguous, segment s at offset s*seg_bytes).  Segment s uses
 * IV_s = iv0 + s (128-bit big-endian add), the "plain64"-style sector IV.
 * A single segment (nseg == 1) is exact single-stream CBC, serial. */
int otc_aes_cbc_encrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                 const otc_aes_key *k, const uint8_t iv0[16], void *stream);
/* _impl: accepted for symmetry; every impl runs the T-table kernels (one
 * serial chain per lane): the persistent claim kernel from 1 GiB (at least
 * 1024 segments), the grid kernel below (its workgroups sized so every CU
 * gets chains).  A VALU
 * kernel for this mode lost at every size and was removed (round 6). */
int otc_aes_cbc_encrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                      const otc_aes_key *k, const uint8_t iv0[16], int impl, void *stream);
/* Same, decryption side (fully parallel).  _impl: with a kernel choice --
 * "auto" runs the T-table + bitsliced split from 2 GiB of power-of-two
 * segments and the persistent T-table claim kernel alone from 512 MiB;
 * OTC_IMPL_BITSLICE runs the bitsliced segment claim kernel alone; other
 * segment sizes: T-table. */
int otc_aes_cbc_decrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                 const otc_aes_key *k, const uint8_t iv0[16], void *stream);
int otc_aes_cbc_decrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                      const otc_aes_key *k, const uint8_t iv0[16], int impl, void *stream);

/* CFB128 over nseg independent segments of seg_bytes (multiple of 16) with
 * IV_s = iv0 + s (128-bit BE add) -- the parallel form of the serial CFB
 * chain, like otc_aes_cbc_encrypt_segments.  Encryption keys for both
 * directions.  Encrypt may run in place; decrypt may not. */
int otc_aes_cfb128_encrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                    const otc_aes_key *k, const uint8_t iv0[16], void *stream);
int otc_aes_cfb128_encrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                         const otc_aes_key *k, const uint8_t iv0[16], int impl, void *stream);
int otc_aes_cfb128_decrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                    const otc_aes_key *k, const uint8_t iv0[16], void *stream);
int otc_aes_cfb128_decrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                         const otc_aes_key *k, const uint8_t iv0[16], int impl, void *stream);

/* CFB128 decryption (parallel): P_i = C_i ^ E(C_{i-1}), C_{-1} = iv;
 * nbytes % 16 == 0; encryption key.  _impl: with a kernel choice (the plain
 * form is OTC_IMPL_AUTO: the T-table + bitsliced split from 2 GiB, the
 * persistent T-table claim kernel from 512 MiB, like ECB encryption). */
int otc_aes_cfb128_decrypt(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                           const uint8_t iv[16], void *stream);
int otc_aes_cfb128_decrypt_impl(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                const uint8_t iv[16], int impl, void *stream);

/* ---- batched CTR: many independent messages in ONE launch -----------------
 * The serving shape (packets, sectors, objects of a few KiB, each with its own
 * key and counter): one launch per message is launch-bound (µs each) and far
 * from the >> 256 workgroups the chip needs.  Here the work unit is a tile of
 * `tile_blocks` 16-byte blocks of one message (64, 128 or 256 = one wave x 1,
 * 2 or 4 blocks per lane: small messages waste less of a small tile, large
 * tiles hide more LDS latency); every array below is DEVICE memory:
 *   msgs[m]        message descriptor (device addresses, length, key index,
 *                  initial 128-bit big-endian counter as two numeric halves)
 *   keys[k]        expanded encryption keys (all with `nr` rounds)
 *   tile_msg[t]    message of tile t          } from otc_ctr_batch_plan()
 *   tile_first[m]  first tile of message m    }
 * in == out (in place) is allowed per message; distinct messages must not
 * overlap.  Messages of 0 bytes have no tiles. */
#define OTC_BATCH_TILE_BLOCKS 256 /* default and largest tile */
typedef struct {
    uint64_t in;      /* device address of the input */
    uint64_t out;     /* device address of the output */
    uint64_t nbytes;
    uint64_t ctr_hi;  /* initial counter, bytes 0..7 as a big-endian number */
    uint64_t ctr_lo;  /* bytes 8..15 */
    uint32_t key;     /* index into keys[] */
    uint32_t align;   /* 0: tiles start at the message's first block.
                         OTC_BATCH_ALIGNED | shift: counter-aligned tiles,
                         shift = ctr_lo mod tile_blocks, so every tile
                         starts at a counter multiple of tile_blocks (the first
                         tile is partial) and rounds 1-2 are mostly computed
                         once per tile (counter-mode caching: 133 instead of
                         160 LDS lookups per AES-128 block) -- for messages of
                         many tiles */
} otc_ctr_msg;
#define OTC_BATCH_ALIGNED 0x80000000u

/* Host planner: fills tile_msg (may be NULL to only count) and tile_first for
 * host copies of the descriptors (honouring each message's `align` word);
 * returns the number of tiles. */
uint64_t otc_ctr_batch_plan(const otc_ctr_msg *msgs, size_t nmsg, int tile_blocks, uint32_t *tile_msg,
                            uint64_t *tile_first);

int otc_aes_ctr_batch(const otc_ctr_msg *msgs, const otc_aes_key *keys, const uint32_t *tile_msg,
                      const uint64_t *tile_first, uint64_t ntiles, int tile_blocks, int nr, void *stream);

/* out = a ^ b (the device arc4_crypt combiner). */
int otc_xor(const void *a, const void *b, void *out, size_t nbytes, void *stream);

/* Many independent RC4 streams, one per lane: stream s uses key
 * keys[s*keylen .. +keylen) (device memory) and produces `len` bytes.
 * If `in` is non-NULL: out[s*len + n] = in[s*len + n] ^ ks_s[n], else the raw
 * keystream is written.  `drop` keystream bytes are discarded first
 * (RC4-drop[n]). */
int otc_rc4_multi(const uint8_t *keys, int keylen, size_t nstreams, size_t len, size_t drop,
                  const void *in, void *out, void *stream);

/* rc4.h on the device (rc4_crypt for many states at once): states is a
 * DEVICE array of nstreams `struct rc4_state` (rc4.h, e.g. set up with
 * rc4_init on the host and copied over); stream s continues from states[s],
 * processes len bytes at in + s*len -> out + s*len (in == out allowed), and
 * its state is written back, so calls resume exactly like rc4_crypt. */
int otc_rc4_crypt_batch(void *states, size_t nstreams, size_t len, const void *in, void *out, void *stream);

/* Deterministic pseudo-random fill (synthetic plaintext). */
int otc_fill_random(void *p, size_t nbytes, uint64_t seed, void *stream);

/* 64-bit XOR-fold checksum of a device buffer (nbytes % 8 == 0) into
 * *out_dev (device pointer to one uint64). */
int otc_checksum(const void *p, size_t nbytes, uint64_t *out_dev, void *stream);

/* Clock probe: a one-wave kernel on `stream` that sleeps `delay_s`, then
 * measures the shader clock over `window_s` seconds of real time; run it on a
 * side stream beside a workload.  out_dev[0] = shader cycles, out_dev[1] =
 * 100 MHz ticks, so GHz = 0.1 * out[0] / out[1]. */
int otc_clock_probe(uint64_t *out_dev, double delay_s, double window_s, void *stream);

/* ---- device memory / sync helpers (so C harnesses need no HIP headers) --- */
void *otc_dev_malloc(size_t nbytes);
void otc_dev_free(void *p);
#define OTC_H2D 0
#define OTC_D2H 1
#define OTC_D2D 2
int otc_memcpy(void *dst, const void *src, size_t nbytes, int kind);
int otc_memset(void *p, int v, size_t nbytes);
/* Elapsed device time of `op` run `iters` times on the default stream,
 * bracketed by hipEvents (kernel-only timing). */
typedef int (*otc_op_fn)(void *arg);
int otc_time_op(otc_op_fn op, void *arg, int iters, double *ms_per_iter);
/* Clock (GHz) the chip holds while running `op` back to back (>= 0.3 s). */
int otc_measure_clock(otc_op_fn op, void *arg, double *ghz);

/* ---- device info ------------------------------------------------------- */
int otc_device_count(void);
int otc_device_cus(int dev);           /* compute units */
int otc_device_clock_khz(int dev);     /* peak shader clock */
int otc_set_device(int dev);
int otc_device_sync(void);
/* A HIP stream for C callers (ordered with the default stream, so events on
 * the default stream bracket work queued on it); NULL on failure. */
void *otc_stream_create(void);
void otc_stream_destroy(void *stream);
/* a and b each wait for the work the other has queued so far (a join point
 * for work split by hand over two streams) */
int otc_stream_join(void *a, void *b);

/* ---- L3 engine: host-memory streaming pipeline -----------------------------
 * Encrypt/decrypt a HOST buffer through one GPU with a pinned staging ring:
 * H2D(k+1) | kernel(k) | D2H(k-1) on three HIP streams.  `host_in` /
 * `host_out` may be pageable (staged through the pinned ring) or already
 * pinned/registered (copied directly).  chunk_bytes: 0 = default (256 MiB).
 */
typedef struct otc_engine otc_engine;

otc_engine *otc_engine_create(int device, size_t chunk_bytes, int depth);
/* flags: OTC_ENGINE_DEFAULT -- the three streams get hardware queues of their
 * own (all-CU-masked streams), so the pipeline overlaps in a process whose
 * other streams (torch, RCCL) fill the 4 pooled queues HIP gives a process;
 * OTC_ENGINE_POOLED_QUEUES -- plain non-blocking streams on the pooled queues
 * (the A/B arm; docs/PERF.md "Round 6"). */
#define OTC_ENGINE_DEFAULT 0
#define OTC_ENGINE_POOLED_QUEUES 1
otc_engine *otc_engine_create_ex(int device, size_t chunk_bytes, int depth, int flags);
void otc_engine_destroy(otc_engine *e);

#define OTC_MODE_ECB 0
#define OTC_MODE_CTR 1
#define OTC_MODE_CBC_DEC 2
#define OTC_MODE_XOR 3

typedef struct {
    double total_ms;      /* wall time of the whole call */
    double kernel_ms;     /* sum of kernel times (hipEvent, kernel stream) */
    double h2d_ms, d2h_ms; /* sum of copy times (hipEvent, copy streams) */
    double host_stage_ms; /* host memcpy into / out of the pinned ring (pageable callers) */
    size_t bytes;
    int chunks;
    int numa_node;        /* node of the pinned ring (-1: unknown / OTC_NUMA=0) */
} otc_stream_stats;

int otc_engine_run(otc_engine *e, int mode, const void *host_in, void *host_out, size_t nbytes,
                   const otc_aes_key *k, const uint8_t iv_or_ctr[16], uint64_t block_offset,
                   int impl, otc_stream_stats *stats);

/* NUMA placement (csrc/cpu/numa.c): the GPU's node from sysfs (-1 unknown);
 * the engine allocates its pinned ring there.  otc_engine_staging returns the
 * ring's input slot (NULL until a pageable run allocated it) so tests can
 * check where its pages live (otc_numa_node_of_addr in otc_numa.h). */
int otc_device_numa_node(int dev);
int otc_engine_numa_node(const otc_engine *e);
const void *otc_engine_staging(const otc_engine *e, int slot);

/* Where a pointer lives: pageable host memory, pinned host memory, or device
 * memory (decides between the kernels and the host pipeline). */
#define OTC_PTR_HOST 0
#define OTC_PTR_PINNED 1
#define OTC_PTR_DEVICE 2
int otc_ptr_kind(const void *p);

/* Pin / unpin an existing host range (hipHostRegister) so the engine copies
 * it without staging. */
int otc_host_register(void *p, size_t nbytes);
int otc_host_unregister(void *p);
void *otc_host_alloc_pinned(size_t nbytes);
void otc_host_free_pinned(void *p);

/* ---- L4 multi-GPU (single process, RCCL over xGMI) -----------------------
 * Shard one host-resident CTR/ECB/CBC-dec stream over `ngpus` devices
 * (strategy 0 with OTC_SHARE_GPUS=1: `ngpus` logical shards mapped onto the
 * visible devices round-robin, to rehearse N shards on fewer GPUs).
 * strategy 0 = direct ingest (each GPU streams its own shard from pinned host
 * memory, engine pipeline per GPU, one host thread per GPU);
 * strategy 1 = RCCL root scatter/gather (root H2D, ncclScatter over xGMI,
 * per-GPU kernel, ncclGather, root D2H), chunked.
 * CBC decryption shards receive a 16-byte halo (the previous shard's last
 * ciphertext block).  Results are byte-identical to the 1-GPU path.
 */
typedef struct {
    double total_ms;
    double gbps;
    int ngpus;
    int strategy;
    int numa_nodes_used; /* strategy 0: distinct NUMA nodes the shard threads ran on */
} otc_multi_stats;

int otc_multi_run(int ngpus, int strategy, int mode, const void *host_in, void *host_out,
                  size_t nbytes, const otc_aes_key *k, const uint8_t iv_or_ctr[16], int impl,
                  size_t chunk_bytes, otc_multi_stats *stats);

/* The round plan of strategy 1, a pure function (csrc/cpu/rccl_plan.c, also
 * in the CPU-only library, so the N > 1 plan is tested without GPUs): the
 * stream goes in rounds of ngpus pieces of `piece` bytes each (the equal
 * counts ncclScatter / ncclGather need); the last round is zero-padded.
 * Piece (r, g) covers stream bytes [off, off + bytes) -- bytes 0 for a piece
 * wholly past the end --, starts at CTR block blk0 = off / 16, and for CBC
 * decryption takes its predecessor block from halo slot `halo` (the 16
 * stream bytes before halo_start(halo)), or the IV when halo < 0. */
typedef struct {
    uint64_t round_off;   /* stream offset of round r */
    uint64_t round_bytes; /* stream bytes in round r (< ngpus * piece: the last round) */
    uint64_t pad_bytes;   /* zero padding of round r's root buffer */
    uint64_t off, bytes;  /* piece (r, g) */
    uint64_t blk0;        /* its first block (CTR counter offset) */
    int64_t halo;         /* CBC decryption: halo slot, -1 = the IV */
} otc_rccl_piece;
uint64_t otc_rccl_nrounds(uint64_t nbytes, int ngpus, uint64_t piece);
/* 0, or OTC_ERR_ARG for ngpus < 1, piece == 0 or a (r, g) out of the plan */
int otc_rccl_plan_piece(uint64_t nbytes, int ngpus, uint64_t piece, uint64_t r, int g, otc_rccl_piece *out);
/* stream offset whose preceding 16 bytes fill halo slot i (clamped to nbytes) */
uint64_t otc_rccl_halo_start(uint64_t nbytes, uint64_t piece, uint64_t i);

/* Free the RCCL communicators / buffers that strategy 1 caches between calls
 * and the per-shard engines of strategy 0 (rebuilt on demand). */
void otc_multi_release(void);
/* Everything the library caches between calls (today: otc_multi_release). */
void otc_release_resources(void);

/* Test hook: make the (after+1)-th runtime allocation from now fail once
 * (device buffers, NUMA-pinned host windows, per-call kernel tables), so the
 * error paths can be exercised on a healthy GPU; after < 0 disarms. */
void otc_fault_inject_alloc(long after);

/* Device-resident multi-GPU CTR: buffers dev_bufs[g] (already on GPU g) hold
 * shard g of `shard_bytes`; all GPUs encrypt in place concurrently with the
 * right counter offsets.  Returns elapsed ms (wall, all GPUs). */
int otc_multi_ctr_resident(int ngpus, void *const *dev_bufs, size_t shard_bytes,
                           const otc_aes_key *k, const uint8_t ctr0[16], int impl,
                           double *elapsed_ms);

/* Library self description / tests */
int otc_bitslice_selftest(int verbose);
const char *otc_build_info(void);
/* JSON object naming the HIP runtime / driver and RCCL versions this process
 * runs on and the mapped libamdhip64 / librccl paths (/proc/self/maps): in a
 * torch process they are torch's bundled copies, elsewhere /opt/rocm's. */
int otc_runtime_info(char *buf, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* OTC_H */
