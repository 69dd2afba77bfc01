/*
 * priskv_crc_gpu.h -- batched value-block CRC on MI355X (gfx950), C ABI.
 *
 * Every checksum computed here is bit-exact with PrisKV's priskv_crc32
 * (server/crc.c:90-109: reflected polynomial 0xEDB88320, init 0, no final
 * xor) applied to each value block on its own.  The reference has no batched
 * or value-block entry point: priskv_crc32 (server/crc.h:37) is its only CRC
 * interface, and these symbols are the new batched form SURVEY.md §8(b)
 * prescribes, declared in a separate header so crc.h and its callers
 * (server/kv.c:314,408, server/rdma.c:764) stay byte-for-byte unchanged.
 *
 * Data layout (the reference's value region, server/memory.h:87-91,
 * server/memory.c:496-508, server/buddy.c:78,165): block i of a batch is the
 * block_size bytes at base + i * block_size.
 *
 * Conventions (the reference's fallible-API style, e.g. server/memory.c:203-210):
 *   return 0 on success or a negative errno:
 *     -EINVAL  bad arguments (NULL pointers with n > 0, block_size 0, ...)
 *     -ENODEV  no usable GPU / the device index does not exist
 *     -ENOMEM  device or pinned-host allocation failed
 *     -EIO     a HIP runtime call failed
 *   Nothing here aborts the process, and there is no CPU fallback: a batch
 *   either runs on the GPU or the call returns an error.
 *
 * Threading: a context is immutable after creation except for the staging
 * buffers of the host-streamed path, which a per-context mutex serialises.
 * The *_dev entry points are asynchronous on the caller's stream and may be
 * called concurrently from any number of threads on one context.
 *
 * Streams are passed as `void *` holding a hipStream_t (NULL = the legacy
 * default stream), so this header does not require the HIP headers.
 *
 * Stream capture: the *_dev calls may be captured into HIP graphs.  A
 * captured call that needs scratch gets a device buffer owned by the graph
 * being captured (freed after the graph and its instantiations are
 * destroyed), so launches of one graph exec are safe back to back; two
 * instantiations of the same captured graph must not run concurrently.
 */
#ifndef PRISKV_CRC_GPU_H
#define PRISKV_CRC_GPU_H

#include <stdint.h>

#if defined(__cplusplus)
extern "C"
{
#endif

typedef struct priskv_crc_ctx priskv_crc_ctx;

/* Create a context on HIP device `device`: uploads the CRC tables (64 KiB
 * LDS images, nibble fold tables, shift matrices) and sizes the persistent
 * grid from the device's CU count.  *out is set only on success.
 * PRISKV_CRC_SEGMENT=0 in the environment at creation turns off the
 * segmentation of few large blocks / extents, PRISKV_CRC_BALANCE=0 the
 * byte-balanced extents split (measurement only). */
int priskv_crc_ctx_create(int device, priskv_crc_ctx **out);
void priskv_crc_ctx_destroy(priskv_crc_ctx *ctx);
int priskv_crc_ctx_device(const priskv_crc_ctx *ctx);

/* Hand the scratch-pool slots `stream` owns back to the context's pool
 * (a slot belongs to the first stream that takes it, by hipStreamGetId;
 * hipStreamPerThread is a different stream on every thread).  Waits for the
 * stream's work first, and frees the scratch of destroyed graphs.  Call it
 * before destroying a stream that ran *_dev calls -- or from a thread about
 * to exit that used hipStreamPerThread -- while no other thread submits to
 * that stream.  Without it the slots of a destroyed stream return to the
 * pool only if the pool was contended when that stream last used them (the
 * library then marked each use's end with its own event); otherwise they
 * stay out of use until ctx_destroy and calls that find no slot allocate
 * per call on their stream.  The library never passes another caller's
 * stream to HIP.  0 / -EINVAL / -ENODEV / -EIO. */
int priskv_crc_stream_release(const priskv_crc_ctx *ctx, void *stream);

/* Device-resident batch: d_base -> nblocks * block_size bytes of device
 * memory; d_out -> uint32_t[nblocks] of device memory.  d_out[i] =
 * priskv_crc32(d_base + i*block_size, block_size).  Asynchronous on `stream`.
 * Any block_size >= 1 and any d_base alignment are accepted.  A 16-byte
 * aligned d_base with block_size a multiple of 1 KiB (or a power of two in
 * [16, 512]) takes the rows (sub-KiB) kernel -- memfile-backed value regions
 * (4 KiB-aligned base, power-of-two size, server/memory.c:221,413-417) always
 * do.  Any other block_size >= 16 (the server's -v takes any size up to
 * 1 MiB, server/server.c:236-244) or base alignment takes the uniform-stride
 * kernel; full rate needs d_base and block_size multiples of 4. */
int priskv_crc32_blocks_dev(const priskv_crc_ctx *ctx, const void *d_base, uint64_t nblocks,
                            uint32_t block_size, uint32_t *d_out, void *stream);

/* Device-resident per-value extents: d_out[i] = priskv_crc32(d_base +
 * d_offsets[i], d_lengths[i]) -- a value of valuelen bytes starting at
 * value_off (priskv_key, server/memory.h:50-51).  d_offsets / d_lengths /
 * d_out are device arrays of n entries.  Asynchronous on `stream`.  With few
 * extents (n <= 8192; PRISKV_CRC_SEG_MAX_EXTENTS) each is split into segments
 * on the device; with a few extents per resident wave the split over the
 * waves is balanced by bytes.  Both need a small scratch allocation: a
 * context pool slot owned by `stream` (the first stream to take a slot keeps
 * it), else one ordered on `stream` (hipMallocAsync); -ENOMEM if that fails. */
int priskv_crc32_ranges_dev(const priskv_crc_ctx *ctx, const void *d_base,
                            const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t n,
                            uint32_t *d_out, void *stream);

/* priskv_crc32_ranges_dev with max_len, an upper bound on every d_lengths[i]
 * that the caller knows on the host (the server holds each valuelen there,
 * server/memory.h:50-51; 0 = unknown, which is priskv_crc32_ranges_dev).  A
 * hint only: every result is exact whatever the lengths, but the launch is
 * chosen from it -- values below 64 KiB are not segmented and the grid is
 * sized by n, so a call of a few small values launches a few workgroups
 * instead of the whole chip, and a bound of 64 KiB or more lets a balanced
 * batch skip the segment plan. */
int priskv_crc32_ranges_dev_bounded(const priskv_crc_ctx *ctx, const void *d_base,
                                    const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t n,
                                    uint64_t max_len, uint32_t *d_out, void *stream);

/* Device-side verify of per-value extents (client-side integrity check):
 * compares priskv_crc32(d_base + d_offsets[i], d_lengths[i]) with
 * d_expected[i] for every i and writes d_status[0] = the number of values
 * that differ and d_status[1] = the smallest such i (UINT64_MAX if none).
 * Replaces copying the whole value pool to the host and memcmp'ing each value
 * (client/benchmark.c:735-761, pypriskv/testing.py:64-66): only 16 bytes of
 * status need to leave the device.  d_status is 2 x uint64_t device memory,
 * written asynchronously on `stream`; d_expected holds the CRCs computed when
 * the values were written (e.g. by this library on the sending buffer). */
int priskv_crc32_verify_dev(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                            const uint32_t *d_lengths, uint64_t n, const uint32_t *d_expected,
                            uint64_t *d_status, void *stream);

/* priskv_crc32_verify_dev with max_len, a host-known upper bound on the
 * lengths (0 = unknown): a launch hint only, exactly as
 * priskv_crc32_ranges_dev_bounded's -- the status is exact whatever the
 * lengths. */
int priskv_crc32_verify_dev_bounded(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                                    const uint32_t *d_lengths, uint64_t n, uint64_t max_len,
                                    const uint32_t *d_expected, uint64_t *d_status, void *stream);

/* Host-resident per-value extents -- the memfile scrub at recovery
 * (server/kv.c:824-875 walks the keys; each live value is valuelen bytes at
 * value_off inside the value region, server/memory.h:50-51).  The kernel
 * reads only the extents' bytes, straight from the host mapping over PCIe
 * (zero-copy): h_base must be registered (priskv_crc_host_register) or
 * pinned, else it is registered for the duration of the call.  h_offsets /
 * h_lengths / h_out are host arrays of n entries; every extent must lie in
 * [0, region_bytes) (-EINVAL otherwise).  Synchronous. */
int priskv_crc32_ranges_host(priskv_crc_ctx *ctx, const void *h_base, uint64_t region_bytes,
                             const uint64_t *h_offsets, const uint32_t *h_lengths, uint64_t n,
                             uint32_t *h_out);

/* Host-resident batch (the RDMA-registered value buffer / the memfile
 * mapping): streams the blocks over PCIe in chunks on several HIP streams,
 * overlapping H2D copies, kernels and the small D2H of results; synchronous.
 * h_out is a host array of nblocks entries.  Pinned (hipHostMalloc) or
 * registered (priskv_crc_host_register) input goes straight to the DMA
 * engines; pageable input is bounced through the context's pinned staging. */
int priskv_crc32_blocks_host(priskv_crc_ctx *ctx, const void *h_base, uint64_t nblocks,
                             uint32_t block_size, uint32_t *h_out);

/* Multi-GPU form of the two host-resident entry points: the blocks (or the
 * extents) are split into nctx contiguous shards, shard g = [g*n/nctx,
 * (g+1)*n/nctx), and each context's device works on its own shard from its
 * own host thread -- each GPU pulls over its own PCIe link, no collective.
 * Returns the first shard's error, if any.  Contexts must be distinct
 * objects (they may share a device). */
int priskv_crc32_blocks_host_multi(priskv_crc_ctx *const *ctxs, int nctx, const void *h_base,
                                   uint64_t nblocks, uint32_t block_size, uint32_t *h_out);
int priskv_crc32_ranges_host_multi(priskv_crc_ctx *const *ctxs, int nctx, const void *h_base,
                                   uint64_t region_bytes, const uint64_t *h_offsets,
                                   const uint32_t *h_lengths, uint64_t n, uint32_t *h_out);

/* SET-completion batcher.  PrisKV finishes a SET when the RDMA READ of the
 * value into its block completes (server/rdma.c:1417-1418 ->
 * server/kv.c:505), per request on each io thread; a launch per value costs
 * more than its CRC, so completions are batched here.  io threads submit
 * (value_off, valuelen, cookie) -- thread-safe and sharded per thread (no
 * shared lock); it blocks only when 8 * max_batch values are already queued.  A worker thread hashes the queue
 * when it holds max_batch values or its oldest value has waited
 * max_delay_us: ONE zero-copy extents pass over h_region (registered at
 * create unless it already is), then cb(arg, cookie, crc, status) for every
 * value from the worker thread -- one submitting thread's values in its
 * submission order -- (status 0, or the pass's -errno with crc 0).  flush blocks until every value submitted
 * before it has been called back; destroy flushes, stops the worker and
 * undoes its registration.  The context must outlive the batcher. */
typedef struct priskv_crc_batch priskv_crc_batch;
typedef void (*priskv_crc_batch_cb)(void *arg, uint64_t cookie, uint32_t crc, int status);
int priskv_crc_batch_create(priskv_crc_ctx *ctx, const void *h_region, uint64_t region_bytes,
                            uint32_t max_batch, uint32_t max_delay_us, priskv_crc_batch_cb cb, void *arg,
                            priskv_crc_batch **out);
int priskv_crc_batch_submit(priskv_crc_batch *b, uint64_t value_off, uint32_t valuelen, uint64_t cookie);
/* n completions at once (one CQ poll's worth): one lock instead of n */
int priskv_crc_batch_submitv(priskv_crc_batch *b, uint64_t n, const uint64_t *value_offs,
                             const uint32_t *valuelens, const uint64_t *cookies);
int priskv_crc_batch_flush(priskv_crc_batch *b);
void priskv_crc_batch_destroy(priskv_crc_batch *b);

/* Page-lock an existing host range (e.g. the mmap'd memfile value region,
 * server/memory.c:351-457) for direct DMA and zero-copy reads by every GPU
 * (portable + mapped), and undo it.  -EEXIST: the range is already registered. */
int priskv_crc_host_register(void *h_base, uint64_t len);
int priskv_crc_host_unregister(void *h_base);

/* GF(2) helpers (host, no GPU needed).  The reference CRC is linear with no
 * affine term (init 0, xorout 0), so
 *   priskv_crc32(A || B) == priskv_crc32_combine(crc(A), crc(B), |B|)
 *   priskv_crc32_shift(c, n) == state c advanced over n zero bytes.      */
uint32_t priskv_crc32_shift(uint32_t crc, uint64_t nbytes);
uint32_t priskv_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* Which host path priskv_crc32 (include/crc.h) folds long inputs with:
 * "vclmul" (VPCLMULQDQ + AVX-512, inputs >= 256 B), "clmul" (PCLMULQDQ,
 * >= 64 B) or "slice8" (tables only).  Chosen once from cpuid; the
 * environment variable PRISKV_CRC_HOST_IMPL=slice8|clmul|vclmul caps it.
 * Shorter inputs always take the slice-by-8 tables.  Diagnostics. */
const char *priskv_crc32_host_impl(void);

/* Deterministic test pattern on the device (benchmarks and parity tests):
 * 64-bit little-endian word i of the region = splitmix64 output
 * mix64(seed + (word_offset + i + 1) * 0x9E3779B97F4A7C15).  Asynchronous. */
int priskv_crc_fill_splitmix_dev(const priskv_crc_ctx *ctx, void *d_dst, uint64_t nbytes,
                                 uint64_t seed, uint64_t word_offset, void *stream);

/* Which kernel family a (d_base, block_size) batch dispatches to on a
 * context with default options: 1 = rows (block a multiple of 1 KiB,
 * 16-byte aligned base: G = 16/32/64 lanes per block; batches of few large
 * blocks are hashed as segments and combined), 3 = sub-KiB power-of-two
 * blocks (16-byte aligned base), 5 = uniform stride (any other block of
 * 16 B up to 9 KiB: rows aligned to each block's end), 2 = extents (the
 * larger such blocks), 4 = generic (blocks
 * below 16 B: one thread per block), 7 = window (a block not a multiple
 * of 1 KiB on a 16-B aligned base, within W - 15 .. W + 48 B of a multiple
 * W of 4 KiB up to 16 KiB -- 4095, 4097, 4100, 8193 B, 4096 B on an odd
 * base -- or, for sizes or bases that are not multiples of 4, up to 48 B
 * above another whole-KiB W up to 6 KiB -- 1025, 2049 B: the rows kernel
 * on each block's 16-B aligned W-byte window, then
 * the few bytes where window and block differ), 6 = head split (a multiple
 * of 4 that is whole 4 KiB chunks of at least 12 KiB plus a 4-64 B head on
 * a 4-byte aligned base, that the window does not take: the rows kernel on
 * the bodies, then the heads' terms; not for a batch of few blocks with
 * bodies of 64 KiB and more, which the extents path segments -- judged for a
 * 256-CU device).  The exact kernels a given context launches, few-block
 * segmentation included, are reported by
 * priskv_crc32_blocks_plan.  For tests and benchmarks; -EINVAL for invalid
 * arguments. */
int priskv_crc32_blocks_path(const void *d_base, uint64_t nblocks, uint32_t block_size);

/* The kernel plan priskv_crc32_blocks_dev would launch for this batch on
 * this context, as a NUL-terminated description in buf (at most len bytes),
 * e.g. "crc_rows_kernel<G=64,CH=4,NBUF=3,nt,pipelined-fold,nibble-fold,
 * progress-priority 3,xcd-weighted 31:29>".  It reflects the context's
 * options (PRISKV_CRC_SEGMENT / _SPLIT / _XCD_WEIGHTS and the XCD probe).
 * Benchmarks and diagnostics; -EINVAL for invalid arguments. */
int priskv_crc32_blocks_plan(const priskv_crc_ctx *ctx, const void *d_base, uint64_t nblocks, uint32_t block_size,
                             char *buf, uint64_t len);

/* Diagnostic: the read roof of the CRC kernel's access pattern.  Reads
 * nblocks x block_size bytes at d_base with the loads, per-wave ranges and
 * XCD split crc_rows_kernel uses for this block size (block_size a multiple
 * of 4 KiB, d_base 16-byte aligned), without hashing.  For an odd block size
 * that the window mode hashes with 4 KiB-multiple windows (4095, 4097, 4100 B
 * ...; priskv_crc32_blocks_path 7) it reads every block's window -- the
 * W bytes ending at the 16-byte boundary at or after the block's end.  variant 0 runs in the
 * CRC plan's own pipeline depth and occupancy; variants 1 ..
 * 6 in 2, 2, 3, 3, 4, 4 chunks in flight at one / two 8-wave workgroups per
 * CU, variants 7 and 8 in the plan's shape with the CRC kernels' progress
 * priority (modes 1 / 3), so the best variant bounds what HBM gives this
 * pattern.  d_sink: PRISKV_CRC_ROOF_SINK_WORDS uint32 entries; launched
 * wave w stores the XOR of the 32-bit words it read in d_sink[w] (plain
 * stores, other entries untouched), so over a zeroed sink the XOR of all
 * entries is the XOR of the batch's words.  Timing it beside
 * priskv_crc32_blocks_dev on the same region gives the fraction of this
 * pattern's roof the CRC reaches.  Asynchronous on stream; 0, or -EINVAL
 * (also for a batch of more than 2^31 chunks per wave) / -ENODEV / -EIO. */
#define PRISKV_CRC_ROOF_VARIANTS 9
#define PRISKV_CRC_ROOF_SINK_WORDS 8192
int priskv_crc_read_roof_dev(const priskv_crc_ctx *ctx, const void *d_base, uint64_t nblocks,
                             uint32_t block_size, uint32_t variant, uint32_t *d_sink, void *stream);

const char *priskv_crc_version(void);

#if defined(__cplusplus)
}
#endif

#endif /* PRISKV_CRC_GPU_H */
