// crc_gpu.hip -- MI355X (gfx950) value-block CRC kernels + the C-ABI shim
// declared in include/priskv_crc_gpu.h.
//
// Function computed: PrisKV's priskv_crc32 (server/crc.c:90-109) -- reflected
// 0xEDB88320, init 0, no final xor -- over each value block of a batch laid
// out as the reference lays out its value region (block i at base +
// i*block_size: server/memory.h:87-91, server/buddy.c:165).
//
// Hot kernel: crc_rows_kernel (block_size a multiple of 1 KiB).  One wave
// per block.  Per row of 1 KiB the wave issues one fully coalesced
// global_load_dwordx4 (lane l gets bytes [16l, 16l+16)), so a 4 KiB block is
// four back-to-back 1 KiB loads.  Each lane runs a slice-by-4 CRC over its
// 16-byte piece of every row:
//     x = u ^ word;  u = E0[x.b0] ^ E1[x.b1] ^ E2[x.b2] ^ E3[x.b3]
// with the four 256-entry tables of Z_4 ("advance 4 bytes") in LDS.  The
// last word of a row uses a second table set for Z_(4 + 1008): that jumps
// the lane's register straight to its piece of the next row, so the
// row-to-row Horner step costs no extra lookup.  After the block's last row
// lane l holds its partial, still 16*(63-l) bytes short of the block end;
// a per-lane GF(2) bit-matrix (32 columns in VGPRs, one v_bfe_i32 +
// v_bitop3 per bit) advances it, and a DPP/readlane XOR over the wave yields
// the block CRC (linear, no affine term: SURVEY §0.2).
//
// LDS layout (64 KiB): row idx (256 B) = [set A: 8 copies x
// (E0,E1,E2,E3)][set B: same].  In lookup instruction i, lane l reads table
// t = (i + l) & 3 from copy k = (l >> 2) & 7, i.e. dword idx*64 + 4k + t:
// bank (addr/4 mod 32) = 4k + t is a bijection of the 32 lanes of a
// ds_read_b32 lane group for ANY indices -> conflict-free with only 8 copies
// (32 KiB per set) instead of 32.  The byte address idx*256 + 16k + 4t is
// built by ONE v_perm_b32 (byte1 <- x byte t, byte0 <- per-lane constant).
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../../include/priskv_crc_gpu.h"
#include "crc_internal.h"

#define PRV_VERSION "priskv-crc-mi355x 0.1 (gfx950)"

namespace {
#include "crc_device.inc"
} // namespace

// ===========================================================================
// host shim
// ===========================================================================
#define NSTREAM 3
#define NPOOL 8 // scratch slots of the *_dev paths

struct priskv_crc_pool_slot {
    void *p;
    size_t size;
    unsigned long long home; // the one stream that uses the slot (StreamKey)
    pthread_t tid;           // ... and its host thread, for a per-thread stream keyed by handle
    int homed;               // home is set (the slot has been taken once)
    int busy;                // taken by a call in flight on the host
    int armed;               // ev was recorded after the slot's last use (pool contended)
    int plain;               // p came from hipMalloc (scratch_alloc), not the stream-ordered pool
    hipEvent_t ev;           // the library's own event (created on first need)
};

struct priskv_crc_ctx {
    int device;
    int num_cus;
    int plan_wgs_per_cu[16];   // resident workgroups per CU of each rows-kernel plan
    uint32_t plan_xw[16];      // rows-kernel split per plan: (even << 16) | odd XCD weight, 0 = equal
    int segment;               // split few large blocks / extents into segments (PRISKV_CRC_SEGMENT=0: off)
    int split;                 // rows kernel split mode for few blocks per wave (PRISKV_CRC_SPLIT=0: off)
    int balance;               // byte-balanced extents split (PRISKV_CRC_BALANCE=0: off)
    int head_split;            // rows kernel + head terms for B = h + whole KiB rows (PRISKV_CRC_HEADSPLIT=0: off)
    int window;                // rows kernel on 16-B aligned windows for sizes near 4 KiB multiples (PRISKV_CRC_WINDOW=0: off)
    uint64_t seg_max_extents;  // device-resident lengths: segment calls of at most this many extents
    int xcd_rr;                // the XCD probe found round-robin dispatch: workgroup b on XCD (b + k) % 8 (weights apply)
    uint64_t tile_min_bytes;   // rows batches of at least this many bytes run in block-cyclic tiles
    uint64_t tile_bytes;       // ... of about this many bytes each
    uint32_t *d_lds_image[3];  // 64 KiB each: set B gap for G = 64, 32, 16
    uint32_t *d_fold;          // kFoldSets x 2048 words, set j for G = 1 << j
    uint32_t *d_nibrep[7];     // nibble fold tables for G = 1 << j (j >= 1), 8 x 16 x max(G, 32) words
    uint32_t *d_nib16;         // the extents kernel's: G = 16, width 16 (8 KiB)
    uint32_t *d_small_img[5];  // sub-KiB byte-fold images for G = 1 << j, j = 1..4 (prv_small_image)
    uint32_t *d_sarwate;       // 256 words
    uint32_t *d_zpow;          // kZpowRows x 32 words: columns of Z_(2^k) (segment combine)
    uint32_t *d_rowshift;      // 16 x 4 x 32 words: columns of Z_-p o Z_(256(3-k)) (extents fold)
    uint32_t *d_winimg;        // window mode images for W = 4, 8, 12, 16 KiB (crc_device.inc s_winimg)
    // host-streamed path (guarded by lock)
    pthread_mutex_t lock;
    int stream_ready;
    size_t chunk_bytes;
    hipStream_t streams[NSTREAM];
    void *d_stage[NSTREAM];
    uint32_t *d_stage_out[NSTREAM];
    void *h_bounce[NSTREAM];
    uint32_t *h_out_stage[NSTREAM];
    // host-extent scrub scratch (guarded by lock)
    size_t scrub_cap;
    void *d_scrub; // offsets | lengths | crcs
    hipStream_t aux; // the context's own stream for synchronous host-resident calls
    // scratch pool of the *_dev paths (Scratch below; guarded by pool_lock)
    mutable pthread_mutex_t pool_lock;
    int pool_ready;
    mutable priskv_crc_pool_slot pool[NPOOL];
    // the fused few-extents kernel's counters + partials (zeroed when
    // allocated; the kernel leaves the counters zero; guarded by pool_lock)
    mutable priskv_crc_pool_slot cnt_pool[NPOOL];
    mutable uint64_t pool_calls;     // pooled takes so far (guarded by pool_lock)
    mutable uint64_t pool_last_miss; // pool_calls at the last take that found no slot (0: never)
    mutable uint64_t pool_misses, pool_takeovers; // diagnostics (priskv_crc_cov_pool, test-only build)
    int fused;                 // few extents in one launch (PRISKV_CRC_FUSED=0: the three-launch path)
};

namespace {

struct DevGuard {
    int old = -1;
    bool ok = false;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&old) != hipSuccess)
            old = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DevGuard()
    {
        if (old >= 0)
            (void)hipSetDevice(old);
    }
};

inline int herr(hipError_t e);

// hipLaunchKernel with the kernel's own parameter types.  Its return value is
// this launch's status; hipGetLastError after hipLaunchKernelGGL would also
// report an earlier, unrelated failure on the calling thread.
template <typename... P, typename... A>
int launch_k(void (*k)(P...), dim3 grid, dim3 block, hipStream_t s, A &&...a)
{
    static_assert(sizeof...(P) == sizeof...(A), "one argument per kernel parameter");
    std::tuple<std::decay_t<P>...> t(static_cast<std::decay_t<P>>(a)...);
    return std::apply(
        [&](auto &...v) {
            void *args[] = {(void *)&v...};
            return herr(hipLaunchKernel(reinterpret_cast<const void *>(k), grid, block, args, 0, s));
        },
        t);
}

inline int herr(hipError_t e)
{
    if (e == hipSuccess)
        return 0;
    if (e == hipErrorOutOfMemory)
        return -ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice)
        return -ENODEV;
    if (e == hipErrorHostMemoryAlreadyRegistered)
        return -EEXIST;
    return -EIO;
}

// Scratch for one *_dev call.  Outside stream capture it comes from the
// context's pool, which saves the stream-ordered alloc/free pair (~6 us of
// host time per call, profiles/r01/host_cost_r4k.json).  A slot belongs to
// the first stream that takes it (StreamKey: hipStreamPerThread is a
// different owner on every thread) and only that stream takes it again, so
// stream order alone puts its previous use first: no event while every
// stream finds a slot.  The library passes no stream to HIP but the one its
// caller handed it in the current call.
//
// Takeover (more streams than slots).  A take that finds no free slot of its
// stream and none unowned marks the pool contended; from then on, until
// kArmCalls pooled takes pass without another miss, each release records the
// slot's own event on the releasing stream before it frees the slot ("armed")
// -- the ~5 us marker rounds 1-3 paid on every call (1 x 256 MiB 54.7 ->
// 49.9 us without it, profiles/r04/pool_event/), now paid only under
// contention.  A stream with no slot takes over a free slot whose armed event
// has completed (hipEventQuery on the library's own event: every use of the
// slot is finished, whether its stream still exists, was destroyed with work
// in flight, or is being captured on another thread).  An unarmed slot of
// another stream is never taken: a stream destroyed without
// priskv_crc_stream_release while the pool was uncontended keeps its slots
// until the context is destroyed, and calls that find no slot take a per-call
// hipMallocAsync / hipFreeAsync on their stream -- a smaller pool, never a
// shared slot.  (Round 5 took over any slot whose home handle hipStreamQuery
// did not report busy: a destroyed handle's error read as idle while its work
// could still run, and querying a stream another thread was capturing broke
// that capture.)  Pool calls run in relaxed capture mode, so another thread's
// global-mode capture does not turn them into errors.
//
// While the stream is capturing, the scratch is a plain device allocation
// the captured graph owns (graph_scratch).  Round 5 replaced graph memory
// nodes (hipMallocAsync inside a capture) with it after 6-16 of 1900
// split-mode blocks came back wrong in graphs with memory-node scratch
// (tools/graph_race_probe.py; the two-word finish that failed
// there is now one word, finish_shared in crc_device.inc).
//
// zero: the memory must read as zeros when a call gets it.  Then `slots` is a
// pool whose users leave their slot zeroed (the fused extents kernel's
// counters): a new allocation is cleared once, a reused slot is not.
constexpr int kGraphOwned = -2; // Scratch::slot of a captured call's graph-owned allocation

// Scratch of a call captured into a graph: a hipMalloc'd buffer (allocated in
// relaxed capture mode, so a global-mode capture is not invalidated) tied to
// the graph being captured by a user object, whose destructor runs when the
// graph and every instantiation of it are gone.  Destructors must not call
// HIP, so it queues the buffer; calls outside capture free the queue once it
// holds kDeferBatch buffers or kDeferBytes (hipFree synchronises the device:
// not on every call after a graph is destroyed), and ctx_destroy /
// priskv_crc_stream_release free whatever is queued.  One buffer per captured
// call: launches of one graph exec are ordered, so only two instantiations of
// one graph launched concurrently could share it (documented in the header).
struct DeferredFree {
    void *p;
    int device;
    size_t bytes;
};
pthread_mutex_t g_defer_lock = PTHREAD_MUTEX_INITIALIZER;
std::vector<DeferredFree> g_deferred;
volatile int g_deferred_n = 0;
volatile size_t g_deferred_bytes = 0;
constexpr int kDeferBatch = 16;
constexpr size_t kDeferBytes = 256u << 20;

void graph_scratch_release(void *arg)
{
    DeferredFree *d = static_cast<DeferredFree *>(arg);
    pthread_mutex_lock(&g_defer_lock);
    try {
        g_deferred.push_back(*d);
        g_deferred_n = (int)g_deferred.size();
        g_deferred_bytes = g_deferred_bytes + d->bytes;
    } catch (...) { // out of host memory: leak the buffer rather than call HIP here
    }
    pthread_mutex_unlock(&g_defer_lock);
    delete d;
}

// free the buffers of destroyed graphs (outside capture: hipFree
// synchronises; relaxed mode, so another thread's global-mode capture does
// not make it an error).  force = false: only once the queue is full.
void free_deferred(bool force)
{
    if (!g_deferred_n || (!force && g_deferred_n < kDeferBatch && g_deferred_bytes < kDeferBytes))
        return;
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    std::vector<DeferredFree> todo;
    pthread_mutex_lock(&g_defer_lock);
    todo.swap(g_deferred);
    g_deferred_n = 0;
    g_deferred_bytes = 0;
    pthread_mutex_unlock(&g_defer_lock);
    int old = -1;
    (void)hipGetDevice(&old);
    for (const DeferredFree &d : todo) {
        (void)hipSetDevice(d.device);
        (void)hipFree(d.p);
    }
    if (old >= 0)
        (void)hipSetDevice(old);
    (void)hipThreadExchangeStreamCaptureMode(&mode);
}

// queue a buffer for free_deferred (its hipFree synchronises the device
// first, so every use of the buffer is complete by then)
void defer_free(void *p, int device, size_t bytes)
{
    DeferredFree *d = new (std::nothrow) DeferredFree{p, device, bytes ? bytes : 4};
    if (d)
        graph_scratch_release(d); // (leaks p if even that allocation fails)
}

// Stream-ordered scratch.  While any blocking stream is being captured, HIP
// refuses hipMallocAsync / hipFreeAsync on every stream, relaxed capture mode
// or not (hipErrorStreamCaptureUnsupported; round 6,
// tools/capture_blocking_probe.py); then the call takes a plain hipMalloc
// (the caller is in relaxed mode) and frees it through the deferred queue.
int scratch_alloc(void **p, size_t bytes, hipStream_t s, int *plain)
{
    *plain = 0;
    const hipError_t e = hipMallocAsync(p, bytes, s);
    if (e == hipSuccess)
        return 0;
    if (e == hipErrorOutOfMemory)
        return -ENOMEM;
    if (hipMalloc(p, bytes) != hipSuccess)
        return herr(e);
    *plain = 1;
    return 0;
}

void scratch_free(void *p, int plain, size_t bytes, hipStream_t s, int device)
{
    if (!p)
        return;
    if (!plain && hipFreeAsync(p, s) == hipSuccess)
        return;
    defer_free(p, device, bytes);
}

int graph_scratch(const priskv_crc_ctx *ctx, hipStream_t s, size_t bytes, void **out)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t *deps = nullptr;
    size_t ndeps = 0;
    if (hipStreamGetCaptureInfo_v2(s, &st, &id, &graph, &deps, &ndeps) != hipSuccess ||
        st != hipStreamCaptureStatusActive || !graph)
        return -EIO;
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    if (hipThreadExchangeStreamCaptureMode(&mode) != hipSuccess)
        return -EIO;
    void *p = nullptr;
    int rc = herr(hipMalloc(&p, bytes ? bytes : 4));
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (rc)
        return rc;
    DeferredFree *d = new (std::nothrow) DeferredFree{p, ctx->device, bytes ? bytes : 4};
    hipUserObject_t obj = nullptr;
    if (!d || hipUserObjectCreate(&obj, d, graph_scratch_release, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
        delete d;
        mode = hipStreamCaptureModeRelaxed;
        (void)hipThreadExchangeStreamCaptureMode(&mode);
        (void)hipFree(p);
        (void)hipThreadExchangeStreamCaptureMode(&mode);
        return -ENOMEM;
    }
    if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
        (void)hipUserObjectRelease(obj, 1); // runs the destructor: the buffer goes to the deferred queue
        return -EIO;
    }
    *out = p;
    return 0;
}

// Which stream a pool slot belongs to.  With a HIP runtime that has
// hipStreamGetId (7.1 and later; looked up at run time, since the runtime a
// process loads -- e.g. the one PyTorch ships -- may be older) the stream's
// id, which names one stream for its whole life.  Otherwise the handle, and
// for hipStreamPerThread -- one handle naming a different stream on every
// host thread -- the handle and the thread.  A handle can name a new stream
// after the old one is destroyed; HIP's hipStreamDestroy waits for the
// stream's work before it frees the stream (checked on the box:
// tests/test_gpu_pool_contention.py::test_stream_destroy_waits_for_its_work),
// so the new owner's calls cannot overlap the old one's.
struct StreamKey {
    unsigned long long v = 0;
    bool per_thread = false;
    pthread_t tid{};
};

typedef hipError_t (*StreamGetIdFn)(hipStream_t, unsigned long long *);
StreamGetIdFn stream_get_id_fn()
{
    static StreamGetIdFn fn = [] {
        Dl_info di;
        if (!dladdr(reinterpret_cast<void *>(&hipStreamQuery), &di) || !di.dli_fname)
            return (StreamGetIdFn) nullptr;
        void *h = dlopen(di.dli_fname, RTLD_LAZY | RTLD_NOLOAD);
        StreamGetIdFn f = h ? reinterpret_cast<StreamGetIdFn>(dlsym(h, "hipStreamGetId")) : nullptr;
        if (h)
            dlclose(h); // (RTLD_NOLOAD: drops only this reference)
        return f;
    }();
    return fn;
}

bool stream_key(hipStream_t s, StreamKey *k)
{
    if (StreamGetIdFn f = stream_get_id_fn())
        return f(s, &k->v) == hipSuccess;
    k->v = (unsigned long long)(uintptr_t)s;
    k->per_thread = s == hipStreamPerThread;
    k->tid = pthread_self();
    return true;
}

bool slot_owned_by(const priskv_crc_pool_slot &q, const StreamKey &k)
{
    return q.homed && q.home == k.v && (!k.per_thread || pthread_equal(q.tid, k.tid));
}

// the calling thread in relaxed capture mode for the guard's lifetime
struct RelaxedCapture {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    bool ok;
    RelaxedCapture() : ok(hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess) {}
    ~RelaxedCapture()
    {
        if (ok)
            (void)hipThreadExchangeStreamCaptureMode(&mode);
    }
};

// pooled takes after the last miss during which releases stay armed
constexpr uint64_t kArmCalls = 1024;

struct Scratch {
    const priskv_crc_ctx *ctx;
    hipStream_t s;
    priskv_crc_pool_slot *slots;
    bool zero;
    int slot = -1;
    void *p = nullptr;
    int plain = 0;    // (slot < 0) p came from hipMalloc
    size_t nbytes = 0;
    Scratch(const priskv_crc_ctx *c, hipStream_t st) : ctx(c), s(st), slots(c->pool), zero(false) {}
    Scratch(const priskv_crc_ctx *c, hipStream_t st, priskv_crc_pool_slot *pool_slots, bool zeroed)
        : ctx(c), s(st), slots(pool_slots), zero(zeroed)
    {
    }
    int zero_fill(void *q, size_t bytes)
    {
        const uint64_t nw = bytes / 4;
        const uint32_t grid = (uint32_t)(nw / 256 + 1 < 1024 ? nw / 256 + 1 : 1024);
        return launch_k(crc_zero_kernel, dim3(grid), dim3(256), s, static_cast<uint32_t *>(q), nw);
    }
    // a free slot for the stream with this key (pool_lock held), or -1
    int pick(const StreamKey &key, size_t bytes) const
    {
        // free slots of this stream first, then unowned ones: the smallest
        // that fits, else the largest (grown)
        int fit[2] = {-1, -1}, grow[2] = {-1, -1};
        for (int i = 0; i < NPOOL; i++) {
            const priskv_crc_pool_slot &q = slots[i];
            if (q.busy || (q.homed && !slot_owned_by(q, key)))
                continue;
            const int o = q.homed ? 0 : 1;
            if (q.size >= bytes) {
                if (fit[o] < 0 || q.size < slots[fit[o]].size)
                    fit[o] = i;
            } else if (grow[o] < 0 || q.size > slots[grow[o]].size) {
                grow[o] = i;
            }
        }
        int k = fit[0] >= 0 ? fit[0] : fit[1] >= 0 ? fit[1] : grow[0] >= 0 ? grow[0] : grow[1];
        if (k >= 0)
            return k;
        // none: the pool is contended; take over a free slot whose armed
        // event has completed (its last use is finished)
        ctx->pool_last_miss = ctx->pool_calls;
        ctx->pool_misses++;
        for (int i = 0; i < NPOOL; i++) {
            const priskv_crc_pool_slot &q = slots[i];
            if (!q.busy && q.armed && q.ev && hipEventQuery(q.ev) == hipSuccess) {
                ctx->pool_takeovers++;
                return i;
            }
        }
        return -1;
    }
    int get(size_t bytes)
    {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusActive;
        const bool capt_ok = hipStreamIsCapturing(s, &cs) == hipSuccess;
        if (capt_ok && cs == hipStreamCaptureStatusActive) {
            if (int rc = graph_scratch(ctx, s, bytes, &p))
                return rc;
            slot = kGraphOwned;
            return zero ? zero_fill(p, bytes) : 0; // a kernel node: every replay starts from zeros
        }
        RelaxedCapture relaxed;
        if (capt_ok && cs == hipStreamCaptureStatusNone)
            free_deferred(false);
        StreamKey key;
        if (ctx->pool_ready && capt_ok && cs == hipStreamCaptureStatusNone && stream_key(s, &key)) {
            pthread_mutex_lock(&ctx->pool_lock);
            ctx->pool_calls++;
            const int k = pick(key, bytes);
            if (k >= 0) {
                slots[k].busy = 1;
                slots[k].homed = 1;
                slots[k].home = key.v;
                slots[k].tid = key.tid;
                slots[k].armed = 0; // an event of an earlier release says nothing about this use
            }
            pthread_mutex_unlock(&ctx->pool_lock);
            if (k >= 0) {
                priskv_crc_pool_slot &q = slots[k];
                int rc = 0;
                if (q.size < bytes) {
                    size_t cap = 64u << 10;
                    while (cap < bytes)
                        cap *= 2;
                    // after the slot's last use: same stream, or a completed armed event
                    scratch_free(q.p, q.plain, q.size, s, ctx->device);
                    q.p = nullptr;
                    q.size = 0;
                    if (!(rc = scratch_alloc(&q.p, cap, s, &q.plain)))
                        q.size = cap;
                    if (!rc && zero && (rc = zero_fill(q.p, cap)))
                        q.size = 0; // not known zero: the next user reallocates (and frees q.p)
                }
                if (rc) {
                    pthread_mutex_lock(&ctx->pool_lock);
                    q.busy = 0;
                    pthread_mutex_unlock(&ctx->pool_lock);
                    return rc;
                }
                slot = k;
                p = q.p;
                return 0;
            }
        }
        nbytes = bytes;
        int rc = scratch_alloc(&p, bytes, s, &plain);
        if (!rc && zero)
            rc = zero_fill(p, bytes);
        return rc;
    }
    // after the call's work is enqueued on s
    int release()
    {
        if (slot == kGraphOwned) // the captured graph frees it
            return 0;
        if (slot < 0) {
            RelaxedCapture relaxed;
            scratch_free(p, plain, nbytes, s, ctx->device);
            p = nullptr;
            return 0;
        }
        priskv_crc_pool_slot &q = slots[slot];
        pthread_mutex_lock(&ctx->pool_lock);
        const bool arm = ctx->pool_last_miss && ctx->pool_calls - ctx->pool_last_miss < kArmCalls;
        pthread_mutex_unlock(&ctx->pool_lock);
        bool armed = false;
        if (arm) { // contended: mark this use's end (the slot is still busy, so nobody takes it meanwhile)
            RelaxedCapture relaxed;
            if (!q.ev && hipEventCreateWithFlags(&q.ev, hipEventDisableTiming) != hipSuccess)
                q.ev = nullptr;
            armed = q.ev && hipEventRecord(q.ev, s) == hipSuccess;
        }
        pthread_mutex_lock(&ctx->pool_lock);
        q.armed = armed;
        q.busy = 0;
        pthread_mutex_unlock(&ctx->pool_lock);
        slot = -1;
        p = nullptr;
        return 0;
    }
};

inline bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }

enum Path {
    PATH_ROWS = 1,
    PATH_EXTENTS = 2,
    PATH_SMALL = 3,
    PATH_GENERIC = 4,
    PATH_STRIDE = 5,
    PATH_HEAD = 6,
    PATH_WINDOW = 7
};

int choose_path(const void *d_base, uint32_t block_size)
{
    const bool aligned = ((uintptr_t)d_base & 15) == 0;
    if (aligned && block_size % PRV_ROW_BYTES == 0)
        return PATH_ROWS;
    if (aligned && is_pow2(block_size) && block_size >= 16 && block_size <= 512)
        return PATH_SMALL;
    if (block_size >= 16)
        return PATH_STRIDE;
    return PATH_GENERIC;
}

int log2u(uint32_t v)
{
    int l = 0;
    while ((1u << l) < v)
        l++;
    return l;
}

int launch_generic(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t n, uint64_t stride,
                   uint32_t len_const, const uint64_t *offs, const uint32_t *lens, uint32_t *out,
                   hipStream_t s)
{
    uint64_t want = (n + 255) / 256;
    uint32_t grid = (uint32_t)(want < (uint64_t)ctx->num_cus * 8 ? want : (uint64_t)ctx->num_cus * 8);
    if (grid == 0)
        grid = 1;
    return launch_k(crc_generic_kernel, dim3(grid), dim3(256), s, base, n, stride, len_const, offs, lens,
                    ctx->d_sarwate, out);
}

constexpr int kNbuf = 2;  // register pipeline depth (chunks) of the extents kernel
constexpr int kAux = 2;   // cache policy of the streaming loads: nt
constexpr int kExtRows = 2; // rows per chunk of the extents kernel (tools/ranges_explore)
// extents kernel: nibble fold + row apply (bit 0), masks only where needed
// (bit 1).  Two shapes (profiles/r01/prio/ranges_prio_16w_*.log): two 8-wave workgroups per CU
// (kExtOpt), and for calls with many extents per wave one 16-wave workgroup
// per CU with progress-priority mode 3 (kExtOptMany: bits 8-9 and 10; the
// progress slots do not fit beside two 80 KiB table sets in 160 KiB of LDS).
// Many small values gain 5-7 %; a few large extents per wave lose 2-4 % in
// the 16-wave shape, so they keep the first.  In the 16-wave shape each wave
// sizes its chunks (8, 4 or 2 rows) from its own extents (bit 14; scattered
// values of 2-4 blocks +5-8 %, tools/ranges_explore, profiles/r03/ranges/).
constexpr int kExtOpt = 3;
constexpr int kExtOptMany = 3 | (3 << 8) | 1024 | 16384;
constexpr uint64_t kExtManyPerWave = 32; // extents per resident wave for kExtOptMany
constexpr int kExtWaves = kWaves;         // kExtOpt's shape: waves per workgroup ...
constexpr int kExtWgPerCu = 2;            // ... and workgroups per CU (the same 16 waves per CU)
static_assert(ext_waves(kExtOpt) == kExtWaves && ext_waves(kExtOptMany) == kExtWaves * kExtWgPerCu,
              "both extents shapes hold 16 waves per CU");

// many: the 16-wave shape (unless PRISKV_CRC_PRIO=0); seg: segmented items;
// bal: byte-balanced split over prefix = the per-tile costs (two 8-wave shape)
int launch_ext_kernel(const priskv_crc_ctx *ctx, bool seg, bool many, bool bal, hipStream_t s, const uint8_t *abase,
                      uint64_t n, const uint64_t *offs, const uint32_t *lens, uint64_t shift, uint64_t stride,
                      uint32_t len_const, uint32_t *out, const uint32_t *prefix, const uint8_t *shifts,
                      const uint32_t *zpow, uint32_t *sub)
{
    const uint32_t *img = ctx->d_lds_image[0], *nib = ctx->d_nib16, *rs = ctx->d_rowshift;
    void *args[] = {(void *)&abase, (void *)&n,   (void *)&offs, (void *)&lens,   (void *)&shift,
                    (void *)&stride, (void *)&len_const, (void *)&img, (void *)&nib, (void *)&rs,
                    (void *)&out,   (void *)&prefix, (void *)&shifts, (void *)&zpow, (void *)&sub};
    const int waves = many ? kExtWaves * kExtWgPerCu : kExtWaves;
    const uint64_t cap = (uint64_t)ctx->num_cus * (many ? 1 : kExtWgPerCu);
    // segmented: the grid covers every resident wave (the kernel reads the
    // segment count on the device); else one wave per extent up to that
    const uint64_t want = seg ? cap : (n + waves - 1) / waves;
    const uint32_t grid = (uint32_t)(want < cap ? want : cap);
    const void *fn;
    if (seg)
        fn = reinterpret_cast<const void *>(&crc_ranges_kernel<kExtRows, kNbuf, kAux, kExtOpt | 4>);
    else if (bal && !many)
        fn = reinterpret_cast<const void *>(&crc_ranges_kernel<kExtRows, kNbuf, kAux, kExtOpt | 2048>);
    else if (many) // 2-row chunks in every wave: 3-12 % slower on scattered values (profiles/r03/ranges/)
        fn = reinterpret_cast<const void *>(&crc_ranges_kernel<kExtRows, kNbuf, kAux, kExtOptMany>);
    else
        fn = reinterpret_cast<const void *>(&crc_ranges_kernel<kExtRows, kNbuf, kAux, kExtOpt>);
    return herr(hipLaunchKernel(fn, dim3(grid ? grid : 1), dim3(64 * waves), args, 0, s));
}

constexpr int kZpowRows = 48;
static_assert(kZpowRows == kFusedZRows, "the fused kernel keeps every Z_(2^k) row in LDS");

int launch_extents_seg(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t n, const uint64_t *offs,
                       const uint32_t *lens, uint64_t stride, uint32_t len_const, uint32_t *out, hipStream_t s,
                       uint64_t max_len, bool *used);

// extents through the row machinery (any base alignment, any lengths).
// max_len: the longest extent when the host knows it (0: unknown)
int launch_extents(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t n, const uint64_t *offs,
                   const uint32_t *lens, uint64_t stride, uint32_t len_const, uint32_t *out, hipStream_t s,
                   uint64_t max_len = 0)
{
    bool used = false;
    if (int rc = launch_extents_seg(ctx, base, n, offs, lens, stride, len_const, out, s, max_len, &used))
        return rc;
    if (used)
        return 0;
    const uint64_t shift = (uintptr_t)base & 15;
    const uint8_t *abase = base - shift;
    const uint64_t waves = (uint64_t)ctx->num_cus * kExtWgPerCu * kExtWaves;
    const bool many = n >= kExtManyPerWave * waves;
    // a few extents per wave: split by bytes, not counts, when
    // the lengths vary (device arrays) and the tile sums fit one wave's scan
    const uint64_t ntiles = (n + kExtTile - 1) / kExtTile;
    if (ctx->balance && offs && !many && n >= waves && ntiles <= 64ull * kExtTileLanes) {
        Scratch scr(ctx, s);
        if (int rc = scr.get(ntiles * sizeof(uint32_t)))
            return rc;
        uint32_t *tiles = static_cast<uint32_t *>(scr.p);
        int rc = launch_k(crc_ext_cost_kernel, dim3((uint32_t)((ntiles + 3) / 4)), dim3(256), s, lens, n, tiles,
                          ntiles);
        if (!rc)
            rc = launch_ext_kernel(ctx, false, false, true, s, abase, n, offs, lens, shift, stride, len_const, out,
                                   tiles, nullptr, nullptr, nullptr);
        const int frc = scr.release();
        return rc ? rc : frc;
    }
    return launch_ext_kernel(ctx, false, many, false, s, abase, n, offs, lens, shift, stride, len_const, out, nullptr,
                             nullptr, nullptr, nullptr);
}

// ---- rows kernel plans --------------------------------------------------------
// (G lanes per block, CH rows per chunk, workgroups per CU) by block size,
// from the tools/crc_explore sweeps recorded in DESIGN.md §5.  Pipeline depth
// (NBUF = 2) and cache policy (nt) are fixed.

enum PlanId {
    PLAN_4K,           // 4 KiB: G64, CH4, 3 chunks in flight, one chunk == one block, fold pipelined, nibble fold
    PLAN_G64_CH4_NIB,  // 8 KiB: G64 with the nibble fold (every 2 chunks)
    PLAN_G16_CH4_PIPE, // 1 KiB (same two folds)
    PLAN_G16_CH4,      // other multiples of 1 KiB up to 16 KiB
    PLAN_G64_CH4,      // 12 KiB and up (multiples of 4 KiB)
    PLAN_G64_CH4_BIG,  // 256 KiB and up (multiples of 4 KiB)
    PLAN_G64_CH2,
    PLAN_G64_CH1,
    PLAN_SPLIT_DEEP,   // split mode for few large blocks: G64, CH4, 3 chunks in flight, first chunks before the tables
    PLAN_4K_DEEP,      // 4 KiB in batches of >= 1 GiB: the 4 KiB plan with 4 chunks in flight
    NPLANS
};
static_assert(NPLANS <= 16, "priskv_crc_ctx per-plan arrays");
struct Plan {
    int G, CH, NBUF, opt, wg_per_cu;
    uint32_t we, wo; // even:odd XCD weights of the static split
};
// opt = crc_rows_kernel OPT bits: 2 = pipelined fold, 32 = nibble-table fold,
// (m << 8) = progress-priority mode m (profiles/r01/explore_*_prio*.log).
// One workgroup per CU everywhere: the G16 plans gain 3-5 % from it over two
// (profiles/r01/prio/occupancy_*.log).
// Weights: swept per plan (profiles/r01/explore_*_xw*.log, bench_xw_ab.jsonl);
// 31:29 is best or within noise for every plan in bench.py's sustained loop.
// 4 KiB: G64 / CH4 / NBUF3 replaced G32 / CH8 / NBUF2 in round 2 -- finer
// chunks with three in flight keep more bytes in flight while a wave hashes;
// +1.4-2.1 % in the explorer on two boxes, same process, bit-identical
// (profiles/r02/explore_r2e_explore_4k_sweep_{a,b}.log, explore_r2f_4k_{a,b}.log).
// NBUF3 loses 1-3 % at 8 KiB-1 MiB (profiles/r02/explore_r2f_{8k,64k,1m}.log),
// so those keep NBUF2.
// Round 3: the 4 KiB plan requests its first chunks before it loads the LDS
// tables (OPT bit 4): 256 MiB calls 48.4 -> 45.6 us, 64 MiB 16.3 -> 16.1,
// 4 GiB level (0.2 %); the 64 KiB plan gained nothing and lost 4 % on
// segmented 64 MiB calls (profiles/r03/early/).
constexpr int kPrio1 = 1 << 8, kPrio3 = 3 << 8, kEarly = 16;
constexpr Plan kPlans[NPLANS] = {
    {64, 4, 3, 2 | kEarly | 32 | kPrio3, 1, 31, 29}, {64, 4, 2, 32 | kPrio1, 1, 31, 29}, {16, 4, 2, 2 | 32 | kPrio1, 1, 31, 29},
    {16, 4, 2, kPrio1, 1, 31, 29},          {64, 4, 2, kPrio1, 1, 31, 29},      {64, 4, 2, kPrio3, 1, 31, 29},
    {64, 2, 2, 0, 1, 31, 29},               {64, 1, 2, 0, 1, 31, 29},
    {64, 4, 3, kEarly | 32 | kPrio3, 1, 31, 29}, // (4 deep: 1 x 256 MiB +1.8 %, 16 x 16 MiB +3.2 % slower, profiles/r04/split/split_deep_nbuf4_ab.jsonl)
    {64, 4, 4, 2 | kEarly | 32 | kPrio3, 1, 31, 29}};

// 4 KiB blocks in batches of at least this many: four chunks in flight
// instead of three, +0.4-0.5 % at 4 GiB on every one of 6 allocations on two
// boxes (same process, profiles/r04/nbuf4k/), while 256 MiB calls are level
// to 2 % slower (a longer pipeline fill); round 2 measured 4 deep -0.9 % at
// 4 GiB on round 2's code.  5 and 6 deep: level (630.4 / 629.7 / 631.4 us
// per 4 GiB call, medians of 5, profiles/r04/nbuf4k/nbuf_4_5_6_ab.jsonl)
constexpr uint64_t kDeep4kBlocks = 1ull << 18; // 1 GiB

int plan_for(uint32_t bs, uint64_t nblocks = 0)
{
    if (bs == 4096)
        return nblocks >= kDeep4kBlocks ? PLAN_4K_DEEP : PLAN_4K;
    if (bs == 8192)
        return PLAN_G64_CH4_NIB;
    if (bs == 1024)
        return PLAN_G16_CH4_PIPE;
    if (bs <= (16u << 10) && bs % 4096 != 0)
        return PLAN_G16_CH4;
    const uint32_t R = bs / PRV_ROW_BYTES;
    if (R % 4 == 0)
        return bs >= (256u << 10) ? PLAN_G64_CH4_BIG : PLAN_G64_CH4;
    return R % 2 == 0 ? PLAN_G64_CH2 : PLAN_G64_CH1;
}

constexpr int plan_waves(int p) { return (kPlans[p].opt & 1024) ? 16 : kWaves; } // waves per workgroup

template <int G, int CH, int NB, int OPT>
const void *plan_kernel()
{
    return reinterpret_cast<const void *>(&crc_rows_kernel<G, CH, NB, kAux, OPT>);
}

// split: the plan's split-mode instance (plans with one block per wave group
// and an unpipelined fold: plan_splits)
constexpr int kSplitOpt = 64, kMergeOpt = 128;
constexpr bool plan_splits(int p) { return kPlans[p].G == 64 && !(kPlans[p].opt & 2); }

template <int P>
const void *plan_kernel_p(bool split)
{
    constexpr Plan Q = kPlans[P];
    if constexpr (plan_splits(P)) {
        // the few-large-blocks plan merges its parts per workgroup (a lone
        // block has a part in every wave; per-wave atomics elsewhere: the
        // workgroup barrier cost 2 % on 4 Ki x 1 MiB, profiles/r04/split/)
        constexpr int SO = kSplitOpt | (P == PLAN_SPLIT_DEEP ? kMergeOpt : 0);
        if (split)
            return plan_kernel<Q.G, Q.CH, Q.NBUF, Q.opt | SO>();
    }
    return plan_kernel<Q.G, Q.CH, Q.NBUF, Q.opt>();
}

const void *plan_fn(int p, bool split = false)
{
    switch (p) {
    case PLAN_4K: return plan_kernel_p<PLAN_4K>(split);
    case PLAN_G64_CH4_NIB: return plan_kernel_p<PLAN_G64_CH4_NIB>(split);
    case PLAN_G16_CH4_PIPE: return plan_kernel_p<PLAN_G16_CH4_PIPE>(split);
    case PLAN_G16_CH4: return plan_kernel_p<PLAN_G16_CH4>(split);
    case PLAN_G64_CH4: return plan_kernel_p<PLAN_G64_CH4>(split);
    case PLAN_G64_CH4_BIG: return plan_kernel_p<PLAN_G64_CH4_BIG>(split);
    case PLAN_G64_CH2: return plan_kernel_p<PLAN_G64_CH2>(split);
    case PLAN_SPLIT_DEEP: return plan_kernel_p<PLAN_SPLIT_DEEP>(split);
    case PLAN_4K_DEEP: return plan_kernel_p<PLAN_4K_DEEP>(split);
    default: return plan_kernel_p<PLAN_G64_CH1>(split);
    }
}

// Block-cyclic tiles for big batches (crc_rows_kernel `tile`): groups per
// tile, 0 = the contiguous per-wave split.  64 KiB blocks, 1 MiB tiles
// against contiguous ranges, same box (profiles/r02/tiles/lib_runs.jsonl,
// tools/lib_timing): 16 GiB 2.558 / 2.436 ms, 32 GiB 4.888 / 4.874,
// 64 GiB 9.859 / 9.802, 128 GiB 20.04 / 21.38 (+6.7 % for tiles; +5.7 % in
// the explorer on another box, explore_r2r_*).  On some boxes the contiguous
// split already slows down at 64 GiB (explore_r2c_explore_64k_size_*), so
// tiles start there.  PRISKV_CRC_TILE_MIN_GIB / PRISKV_CRC_TILE_KIB move the
// switch and the tile size.
constexpr uint64_t kTileMinBytes = 64ull << 30;
constexpr uint64_t kTileBytes = 1ull << 20;

uint32_t tile_groups(const priskv_crc_ctx *ctx, uint64_t ngroups, uint64_t gstride)
{
    if (ngroups * gstride < ctx->tile_min_bytes)
        return 0;
    const uint64_t t = ctx->tile_bytes / gstride;
    return t ? (uint32_t)(t < (1u << 20) ? t : (1u << 20)) : 1u;
}

// the XCD weights of a split-mode launch over n units: from 32 units per wave
uint32_t split_units_xw(const priskv_crc_ctx *ctx, int p, uint64_t n)
{
    const uint64_t max_wgs = (uint64_t)ctx->num_cus * ctx->plan_wgs_per_cu[p];
    const uint64_t want = (n + kWaves - 1) / kWaves;
    const uint64_t grid = want < max_wgs ? want : max_wgs;
    return n >= 32ull * grid * kWaves ? ctx->plan_xw[p] : 0u;
}

// stride: bytes from block to block (0: bs; more for the head-split bodies).
// split > 1: the split mode (ngroups = blocks; acc: zeroed scratch of
// ngroups 64-bit words, left zero), one launch
int launch_plan(const priskv_crc_ctx *ctx, int p, const uint8_t *base, uint64_t ngroups, uint32_t bs, uint32_t *out,
                hipStream_t s, uint32_t stride = 0, uint32_t split = 1, uint64_t *acc = nullptr)
{
    if (!stride)
        stride = bs;
    const Plan &P = kPlans[p];
    const int gi = P.G == 64 ? 0 : (P.G == 32 ? 1 : 2);
    const uint64_t max_wgs = (uint64_t)ctx->num_cus * ctx->plan_wgs_per_cu[p];
    const uint64_t NW = (uint64_t)plan_waves(p);
    const uint64_t nb_per_group = 64 / P.G;
    const uint64_t cps = bs / ((uint64_t)P.CH * 16u * P.G);
    const uint32_t *img = ctx->d_lds_image[gi];
    const uint32_t *fold = (P.opt & 32) ? ctx->d_nibrep[log2u(P.G)] : ctx->d_fold + log2u(P.G) * 2048;
    const uint32_t *zp = ctx->d_zpow;
    if (split > 1) { // one launch over ngroups * split units (host-checked: < 2^31 chunks per wave)
        uint64_t n = ngroups * split;
        const uint64_t want = (n + NW - 1) / NW;
        const uint32_t grid = (uint32_t)(want < max_wgs ? want : max_wgs);
        uint32_t xw = split_units_xw(ctx, p, n), tile = 0;
        void *args[] = {(void *)&base, (void *)&n,    (void *)&bs,    (void *)&img,   (void *)&fold,
                        (void *)&out,  (void *)&xw,   (void *)&tile,  (void *)&stride, (void *)&split,
                        (void *)&zp,   (void *)&acc};
        return herr(hipLaunchKernel(plan_fn(p, true), dim3(grid), dim3(64 * NW), args, 0, s));
    }
    // the kernel counts a wave's chunks in 32 bits: cap groups per launch
    const uint64_t cap = max_wgs * NW * ((1ull << 31) / cps - 1);
    for (uint64_t done = 0; done < ngroups;) {
        uint64_t n = (ngroups - done < cap) ? ngroups - done : cap;
        const uint64_t want = (n + NW - 1) / NW;
        const uint32_t grid = (uint32_t)(want < max_wgs ? want : max_wgs);
        const uint8_t *b = base + done * nb_per_group * stride;
        uint32_t *o = out + done * nb_per_group;
        // weights move whole groups: only worth it with many groups per wave
        uint32_t xw = n >= 32ull * grid * NW ? ctx->plan_xw[p] : 0u;
        uint32_t tile = tile_groups(ctx, n, nb_per_group * stride);
        uint32_t one = 1;
        uint64_t *none = nullptr;
        void *args[] = {(void *)&b,  (void *)&n,    (void *)&bs,   (void *)&img,    (void *)&fold,
                        (void *)&o,  (void *)&xw,   (void *)&tile, (void *)&stride, (void *)&one,
                        (void *)&zp, (void *)&none};
        if (int rc = herr(hipLaunchKernel(plan_fn(p), dim3(grid), dim3(64 * NW), args, 0, s)))
            return rc;
        done += n;
    }
    return 0;
}

// Few large blocks: the rows kernel splits block GROUPS statically over the
// resident waves, so 1024 x 1 MiB (1024 groups for 2048 waves) leaves half
// the chip idle and 3000 groups run at 3000 / (2 * 2048) = 73 % balance.
// When that balance r / ceil(r) (r = groups per resident wave) is below
// 0.9, each block is hashed as S equal segments (S a power of two, segments
// >= 16 KiB and whole 1 KiB rows), doubling S until the balance is reached,
// and the segment CRCs are combined by crc_combine_segments_kernel.
constexpr uint32_t kMinSegment = 16u << 10;

bool balanced(uint64_t units, uint64_t waves)
{
    const uint64_t c = (units + waves - 1) / waves; // units of the busiest wave
    return units * 10 >= c * waves * 9;
}

uint32_t segments_for(const priskv_crc_ctx *ctx, uint64_t nblocks, uint32_t bs)
{
    const uint64_t waves = (uint64_t)ctx->num_cus * kWaves; // 1 WG/CU: the plans for blocks > 16 KiB
    uint32_t S = 1;
    if (!ctx->segment)
        return S;
    while (!balanced(nblocks * S, waves) && bs / (2 * S) >= kMinSegment && (bs / (2 * S)) % PRV_ROW_BYTES == 0 &&
           bs % (2 * S) == 0)
        S *= 2;
    return S;
}

int launch_rows_plain(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t *out,
                      hipStream_t s, uint32_t stride = 0);

// Split mode (crc_rows_kernel OPT bit 6): a balanced batch with
// fewer than kSplitUnitsPerWave blocks per wave (1 MiB blocks: 2) cannot take
// the XCD weights, which move whole blocks.  Cut each block into S units
// (S a power of two, units of whole 4 KiB chunks and >= kSplitMinUnit) until
// there are kSplitUnitsPerWave units per wave, and the weights apply to
// units; parts of blocks combine inside the launch.  1 = no split (the
// weights already apply or are off, no such S, PRISKV_CRC_SPLIT=0).
constexpr uint64_t kSplitUnitsPerWave = 32;
constexpr uint32_t kSplitMinUnit = 16u << 10;

uint32_t split_for(const priskv_crc_ctx *ctx, uint64_t nblocks, uint32_t bs)
{
    const int p = plan_for(bs);
    // (block-cyclic tiles win where both apply: batches of >= 64 GiB, or
    // PRISKV_CRC_TILE_MIN_GIB; split plans are G = 64, one block per group)
    if (!ctx->split || !plan_splits(p) || !ctx->plan_xw[p] || bs % 4096 != 0 || tile_groups(ctx, nblocks, bs))
        return 1;
    const uint64_t want = kSplitUnitsPerWave * (uint64_t)ctx->num_cus * ctx->plan_wgs_per_cu[p] * kWaves;
    if (nblocks >= want)
        return 1;
    uint32_t S = 1;
    while (nblocks * S < want && (bs / 4096) % (2 * S) == 0 && bs / (2 * S) >= kSplitMinUnit)
        S *= 2;
    return nblocks * S >= want ? S : 1;
}

// Few large blocks (the count split is unbalanced, segments_for > 1): the
// same split mode instead of segments + a combine kernel or the fused
// kernel, with units down to one 4 KiB chunk, and on the 3-deep plan that
// requests its first chunks before the tables (the 4 KiB plan's edge at
// small calls: DESIGN §6).  Units aim at kSplitUnitsPerWave per wave (the
// XCD weights apply from there) and are accepted from kSplitFewMinPerWave:
// 32 MiB to 256 MiB batches (512 x 64 KiB, 100 x 1 MiB, 1000 x 128 KiB,
// 200 x 512 KiB, 1500 x 64 KiB) then run 13-34 % faster than through
// segments + combine (profiles/r04/split/split_few_units_ab.jsonl), while
// larger ones keep their 32 units (aiming lower, at 4-16 per wave, cost
// 1 x 256 MiB 5 %: split_few_upw_sweep.jsonl).  1 = not applicable (then
// segments as before).
constexpr uint64_t kSplitFewMinPerWave = 4;

uint32_t split_few(const priskv_crc_ctx *ctx, uint64_t nblocks, uint32_t bs)
{
    if (!ctx->split || bs % 4096 != 0)
        return 1;
    const uint64_t waves = (uint64_t)ctx->num_cus * ctx->plan_wgs_per_cu[PLAN_SPLIT_DEEP] * kWaves;
    uint32_t S = 1;
    while (nblocks * S < kSplitUnitsPerWave * waves && (bs / 4096) % (2 * S) == 0)
        S *= 2;
    return nblocks * S >= kSplitFewMinPerWave * waves ? S : 1;
}

int launch_split(const priskv_crc_ctx *ctx, int p, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t S,
                 uint32_t *out, hipStream_t s)
{
    Scratch sc(ctx, s, ctx->cnt_pool, true); // zero at rest: the kernel leaves it zero
    if (int rc = sc.get((size_t)nblocks * 8))
        return rc;
    const int rc = launch_plan(ctx, p, base, nblocks, bs, out, s, 0, S, static_cast<uint64_t *>(sc.p));
    const int frc = sc.release();
    return rc ? rc : frc;
}

// Few extents: the same kernel over segments of each extent.  The segments
// are laid out on the device by crc_seg_plan_kernel (the host never sees
// device-resident lengths); each segment's CRC is shifted to its extent's
// end inside the extents kernel, and crc_seg_reduce_kernel XORs them.  The
// segment-count cap per extent aims at about two segments per resident
// wave; the scratch is stream-ordered like the rows path's.
//
// When.  The two extra launches and the scratch cost several us per call
// (tools/bench_paths.py few): a loss for small values, which one wave
// hashes in a few us, and a large win for big ones (one wave streams only
// ~3.4 GB/s: 32 x 1 MiB 311 -> 23 us, 1 x 256 MiB 70.6 ms -> 97 us;
// profiles/r01/few_values.jsonl).  When the host knows the longest extent
// (one constant length on the blocks path, host arrays on the host scrub),
// segment when the batch is unbalanced and that length is at least
// kSegMinLen.  Device-resident lengths are unknown, so the rule uses the
// count: at most kSegMaxExtents extents, twice the resident waves.  On the
// current segmented path (one segment size per call) PrisKV-shaped values
// at 8192 cost small values ~11 us (4 KiB blocks: 29 -> 40 us) and save
// 0.65-0.75 ms on MiB values (1 MiB blocks, 4096: 1864 -> 1214 us, 8192:
// 3252 -> 2498 us; 64 KiB blocks 209 -> 191 us); at 16384 the gain shrinks
// to 5 % and small values lose 26 us (profiles/r01/seg_limit_r4g.jsonl).
// KV-cache values are the large kind.
// PRISKV_CRC_SEG_MAX_EXTENTS moves the threshold (0 = never for device lengths).
constexpr uint64_t kSegMaxExtents = 8192;
constexpr uint64_t kSegPerWave = 8; // full segments per resident wave (tools/bench_paths.py few / ranges)
constexpr uint32_t kSegMinLen = 64u << 10;
// progress priority off in the fused kernel: 1 x 256 MiB 49.7 us vs 50.7 with
// mode 3, 4096 small values 7.6 vs 7.7 us (profiles/r02/fused/ktrace_shapes_*)
constexpr int kFusedPrio = 0;
constexpr uint64_t kFusedUnitsPerWave = 32; // with XCD weights (fused_xw)
constexpr uint32_t kFusedMinShift = 10;     // ... segments of at least 1 KiB

// one segment size per call (crc_seg_plan_kernel / the fused kernel): about
// kSegPerWave full segments per resident wave, so the count split of
// segments is a byte split; at most n + target segments, and segment
// distances stay below 2^16
uint64_t seg_target(const priskv_crc_ctx *ctx)
{
    const uint64_t waves = (uint64_t)ctx->num_cus * kExtWgPerCu * kExtWaves;
    return std::min<uint64_t>(kSegPerWave * waves, 32768);
}

// does an extents call take the segmented path?  max_len: the longest
// extent when the host knows it (0: device-resident lengths)
bool extents_segmented(const priskv_crc_ctx *ctx, uint64_t n, uint64_t max_len)
{
    const uint64_t waves = (uint64_t)ctx->num_cus * kExtWgPerCu * kExtWaves;
    if (!ctx->segment || n == 0 || n > (uint64_t)kSegPlanThreads * kSegPlanPerThread)
        return false;
    return max_len ? !(max_len < kSegMinLen || balanced(n, waves)) : n <= ctx->seg_max_extents;
}

// the fused few-extents kernel, one launch (n <= kFusedMaxExtents): the plan
// inside every workgroup; extents shared by workgroups finish through one
// zero-at-rest 64-bit word each (count, XOR) that the kernel leaves zero
int launch_fused(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t n, const uint64_t *offs,
                 const uint32_t *lens, uint64_t stride, uint32_t len_const, uint32_t *out, hipStream_t s)
{
    static_assert(kFusedMaxExtents == (uint64_t)kSegPlanThreads * kSegPlanPerThread, "one extent limit");
    if (n == 0 || n > kFusedMaxExtents)
        return -EINVAL;
    const uint32_t grid = (uint32_t)ctx->num_cus;
    Scratch sc(ctx, s, ctx->cnt_pool, true);
    if (int rc = sc.get((size_t)kFusedMaxExtents * 8))
        return rc;
    uint64_t *acc = static_cast<uint64_t *>(sc.p);
    const uint64_t sh = (uintptr_t)base & 15;
    const uint8_t *abase = base - sh;
    const uint32_t *lens_or_null = offs ? lens : nullptr;
    // XCD weights (fused_xw): segments of >= 1 KiB, about kFusedUnitsPerWave per
    // resident wave, so that the weights (whole units) apply to large calls;
    // else about kSegPerWave of >= 16 KiB (round 3)
    // Shape: 16 waves per CU with 2-row chunks 2 deep, whatever the count.
    // Rounds 4-5 ran at most 16 extents -- a lone large value, a few -- on 8
    // waves with 4-row chunks, which streamed 4-8 % faster there
    // (profiles/r04/fused/shape_ab.jsonl).  With round 6's one-word finish
    // the 16-wave shape (and its finer segment target) came out 1-2 % faster
    // for those calls too: 1 x 256 MiB 53.4 -> 52.3 us, 4 x 64 MiB 52.1 ->
    // 51.1, 16 x 2 MiB 14.5 -> 14.4, medians of 12 in one process
    // (profiles/r06/fused/fused_16w_ab.jsonl).
    const int nw = kFusedWaves;
    const uint64_t waves = (uint64_t)ctx->num_cus * nw;
    const uint64_t want = kFusedUnitsPerWave * waves;
    const uint32_t tgt = 1u << (31 - __builtin_clz((uint32_t)std::min<uint64_t>(want, 1u << 30))); // a power of two
    uint32_t ms = kFusedMinShift;
    uint32_t xw = ctx->plan_xw[PLAN_4K];
    // (16 waves: 4- and 8-row chunks lost 6-13 % on a lone 256 MiB value, profiles/r03/fused/)
    const void *fn = reinterpret_cast<const void *>(&crc_ranges_fused_kernel<kExtRows, kNbuf, kAux, kFusedPrio, kFusedWaves>);
    const uint32_t *img = ctx->d_lds_image[0], *nib = ctx->d_nib16, *rs = ctx->d_rowshift, *zp = ctx->d_zpow;
    void *args[] = {(void *)&abase, (void *)&n,   (void *)&offs, (void *)&lens_or_null, (void *)&sh,
                    (void *)&stride, (void *)&len_const, (void *)&img, (void *)&nib, (void *)&rs,
                    (void *)&out,   (void *)&zp,  (void *)&tgt, (void *)&ms, (void *)&acc, (void *)&xw};
    const int rc = herr(hipLaunchKernel(fn, dim3(grid), dim3(64 * nw), args, 0, s));
    const int frc = sc.release();
    return rc ? rc : frc;
}

int launch_extents_seg(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t n, const uint64_t *offs,
                       const uint32_t *lens, uint64_t stride, uint32_t len_const, uint32_t *out, hipStream_t s,
                       uint64_t max_len, bool *used)
{
    *used = false;
    if (!extents_segmented(ctx, n, offs ? max_len : len_const))
        return 0;
    *used = true;
    if (ctx->fused)
        return launch_fused(ctx, base, n, offs, lens, stride, len_const, out, s);
    // PRISKV_CRC_FUSED=0: plan kernel -> extents kernel -> reduce kernel
    const uint64_t target = seg_target(ctx);
    const size_t off_shift = ((n + 1) * 4 + 255) / 256 * 256;
    const size_t off_sub = off_shift + (n + 255) / 256 * 256;
    Scratch sc(ctx, s);
    if (int rc = sc.get(off_sub + (n + target) * 4))
        return rc;
    uint8_t *scr = static_cast<uint8_t *>(sc.p);
    uint32_t *prefix = reinterpret_cast<uint32_t *>(scr);
    uint8_t *shifts = scr + off_shift;
    uint32_t *sub = reinterpret_cast<uint32_t *>(scr + off_sub);
    int rc = launch_k(crc_seg_plan_kernel, dim3(1), dim3(kSegPlanThreads), s, offs ? lens : nullptr, len_const, n,
                      (uint32_t)target, prefix, shifts);
    if (!rc) {
        const uint64_t sh = (uintptr_t)base & 15;
        rc = launch_ext_kernel(ctx, true, false, false, s, base - sh, n, offs, lens, sh, stride, len_const, out, prefix, shifts,
                               ctx->d_zpow, sub);
    }
    if (!rc) {
        const uint32_t grid = (uint32_t)n; // one workgroup per extent (n <= 16384)
        rc = launch_k(crc_seg_reduce_kernel, dim3(grid), dim3(kSegReduceThreads), s, sub, prefix, shifts,
                      offs ? lens : nullptr, len_const, ctx->d_zpow, n, out);
    }
    const int frc = sc.release();
    *used = true;
    return rc ? rc : frc;
}

// few large blocks through the fused kernel up to the wave-planned size (1024 x
// 1 MiB is 3 % faster through rows + combine)
bool fused_blocks(const priskv_crc_ctx *ctx, uint64_t nblocks) { return ctx->fused && nblocks <= kFusedWavePlan; }

int launch_rows(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t *out,
                hipStream_t s)
{
    const uint32_t S = segments_for(ctx, nblocks, bs);
    if (S == 1) {
        const uint32_t sp = split_for(ctx, nblocks, bs);
        return sp > 1 ? launch_split(ctx, plan_for(bs), base, nblocks, bs, sp, out, s)
                      : launch_rows_plain(ctx, base, nblocks, bs, out, s);
    }
    if (const uint32_t sf = split_few(ctx, nblocks, bs); sf > 1)
        return launch_split(ctx, PLAN_SPLIT_DEEP, base, nblocks, bs, sf, out, s);
    // few large blocks: the fused few-extents kernel in one launch (1 x 256 MiB
    // 50 us against 55-57 for rows + combine, 1024 x 1 MiB level: DESIGN §4)
    if (fused_blocks(ctx, nblocks))
        return launch_fused(ctx, base, nblocks, nullptr, nullptr, bs, bs, out, s);
    Scratch sc(ctx, s); // pooled, ordered by events: concurrent calls never share a slot
    if (int rc = sc.get(nblocks * S * sizeof(uint32_t)))
        return rc;
    uint32_t *sub = static_cast<uint32_t *>(sc.p);
    int rc = launch_rows_plain(ctx, base, nblocks * S, bs / S, sub, s);
    if (!rc) {
        const uint32_t r = S > 64 ? S / 64 : 1; // segments per lane (S is a power of two)
        SegCols z;
        prv_shift_columns(z.c[0], bs / S);
        for (int b = 0; b < 6; b++)
            prv_shift_columns(z.c[1 + b], (uint64_t)(bs / S) * r << b);
        const uint64_t want = (nblocks + 3) / 4; // one wave per block
        const uint32_t grid = (uint32_t)(want < (uint64_t)ctx->num_cus * 8 ? want : (uint64_t)ctx->num_cus * 8);
        rc = launch_k(crc_combine_segments_kernel, dim3(grid), dim3(256), s, sub, nblocks, S, r, z, out);
    }
    const int frc = sc.release();
    return rc ? rc : frc;
}

int launch_rows_plain(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t *out,
                      hipStream_t s, uint32_t stride)
{
    if (!stride)
        stride = bs;
    const int p = plan_for(bs, nblocks);
    const uint64_t per = 64 / kPlans[p].G; // blocks per wave group
    const uint64_t head = nblocks - nblocks % per;
    if (head)
        if (int rc = launch_plan(ctx, p, base, head / per, bs, out, s, stride))
            return rc;
    if (head == nblocks)
        return 0;
    // ragged tail (< per blocks): one wave per block
    const uint32_t R = bs / PRV_ROW_BYTES;
    const int pt = R % 4 == 0 ? PLAN_G64_CH4 : (R % 2 == 0 ? PLAN_G64_CH2 : PLAN_G64_CH1);
    return launch_plan(ctx, pt, base + head * (uint64_t)stride, nblocks - head, bs, out + head, s, stride);
}

// ---- head-split blocks -------------------------------------------------------
// A block size B that is a multiple of 4 with a small remainder over whole
// KiB rows, B = h + body (h = B mod 1 KiB, 4 <= h <= kHeadMax, body >= 1
// KiB), on a 4-byte aligned base: the rows kernel hashes the bodies in place
// (stride B, 4-byte aligned loads stream at full rate) and crc_head_kernel
// adds each head's term Z_body(crc(head)).  A 4096-B value with a 4-B
// trailer, 4100 B, thus runs on the 4 KiB plan instead of the stride
// kernel's 9 rows of 512 B for 4100 (12 % of them padding).  The bodies run
// unsegmented, so a batch of few large blocks -- one the extents path would
// segment: bodies of at least kSegMinLen and a count split that is not
// balanced over the rows kernel's waves -- keeps the stride / extents paths,
// which hand it to the fused kernel (whatever the body: 1023 KiB bodies cannot
// be halved into whole-KiB segments, and one wave streams ~3.4 GB/s).
// Round 5: the window mode takes heads of up to 48 B below 16 KiB first, and
// the head split now runs only on bodies that are whole 4 KiB chunks of at
// least 12 KiB -- against the stride / extents kernels (same process, ~4 GB
// per call, profiles/r05/window/headsplit_*.jsonl) it gained 16436 B +4-7 %,
// 1 MiB + 4 +6-7 %, 64 KiB + 4 +2-3 %, 12340 B +2 %, but lost 1088 B -19 %,
// 17412 B -22 % (1 KiB and 17 KiB bodies: the G16 and one-row plans), 8244
// B -4-6 % and 4148 / 9220 B -2 %.
// PRISKV_CRC_HEADSPLIT=0 turns it off.  ctx = nullptr: a default context on
// a device of kNominalCus CUs (priskv_crc32_blocks_path).
constexpr int kNominalCus = 256; // MI355X
constexpr uint32_t kHeadMinBody = 12u << 10;
bool head_split(const priskv_crc_ctx *ctx, const void *base, uint64_t nblocks, uint32_t bs)
{
    const uint32_t h = bs % PRV_ROW_BYTES, body = bs - h;
    if (!((!ctx || ctx->head_split) && bs % 4 == 0 && ((uintptr_t)base & 3) == 0 && h >= 4 && h <= kHeadMax &&
          body >= kHeadMinBody && body % 4096 == 0))
        return false;
    const bool seg = ctx ? ctx->segment != 0 : true;
    const uint64_t waves = (uint64_t)(ctx ? ctx->num_cus : kNominalCus) * kWaves;
    return !seg || body < kSegMinLen || balanced(nblocks, waves);
}

int launch_head_split(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t *out,
                      hipStream_t s)
{
    const uint32_t h = bs % PRV_ROW_BYTES, body = bs - h;
    if (int rc = launch_rows_plain(ctx, base + h, nblocks, body, out, s, bs))
        return rc;
    HeadCols z;
    prv_shift_columns(z.c, body);
    const uint64_t want = (nblocks + 255) / 256;
    const uint32_t grid = (uint32_t)(want < (uint64_t)ctx->num_cus * 8 ? want : (uint64_t)ctx->num_cus * 8);
    return launch_k(crc_head_kernel, dim3(grid), dim3(256), s, base, nblocks, bs, h, ctx->d_sarwate, z, out);
}

// ---- window blocks -------------------------------------------------------------
// A block size B within [W - 15, W + 48] of a whole number W of KiB (W <= 16
// KiB; window_bytes says which) that is not a multiple of 1 KiB on a 16-B
// aligned base -- 4095, 4097, 8193, 1025, 2049 B, 4100 B, 4096 B at base +
// 1: the rows kernel hashes each block's window, the W bytes that end at
// the first 16-B boundary at or after the block's end (crc_rows_kernel OPT
// bit 13: aligned rows at W's plan), each CRC corrected for the bytes where
// window and block differ when the wave stores 64 of them (crc_device.inc
// s_winimg).  It goes before the head split, which keeps the
// multiples of 4 it does not reach (heads of 49-64 B, W above 16 KiB).
// PRISKV_CRC_WINDOW=0 turns it off (the head split, stride kernel or
// extents path).
constexpr uint32_t kWinMaxBytes = 16u << 10, kWinOver = 48;
constexpr uint32_t kStrideMax = 9u << 10; // the stride / extents kernels' boundary (stride_to_extents)
constexpr int kWinImages = (int)(kWinMaxBytes / 1024);
constexpr int kWinOpt = 8192;

uint32_t window_bytes(const priskv_crc_ctx *ctx, const void *base, uint64_t nblocks, uint32_t bs)
{
    const uint32_t W = (uint32_t)(((uint64_t)bs + 15) / 1024 * 1024); // W - 15 <= bs
    (void)nblocks; // (blocks this small are never segmented: kSegMinLen)
    static_assert(kWinMaxBytes + kWinOver < kSegMinLen, "window sizes are never segmented");
    if ((ctx && !ctx->window) || W == 0 || W > kWinMaxBytes || bs > W + kWinOver)
        return 0;
    // W not a multiple of 4 KiB (the G = 16 plans): only up to 6 KiB, only
    // for sizes or bases that are not multiples of 4 (where the stride
    // kernel funnel-shifts), and there only above W (where the stride kernel
    // pads a whole extra row) or, for W = 1 KiB, below it.  Per ~4 GB call
    // (profiles/r05/window/g16_*.jsonl, odd_sweep*.jsonl): 1025 B 843 -> 693
    // us, 2049 B 791 -> 687, 3073 B 673 -> 656, 1023 B 713 -> 682, 1041 /
    // 2065 / 3089 B +10 / +10 / +2 %; but multiples of 4 (1040, 2056, 3076,
    // 5124 B: the stride kernel's aligned loads) 1-7 % slower, 2047 / 3071 /
    // 6143 B level, 2048 B on base + 1 643 -> 676, 7169 B -1 %, and from 9
    // KiB the extents kernel is faster (9217 B 644 against 649, 15361 B 602
    // against 633)
    if (W % 4096 != 0) {
        const bool odd = (((uintptr_t)base | bs) & 3u) != 0;
        if (!odd || W > 6144 || (W > 1024 && bs <= W) || (W == 1024 && bs == W))
            return 0;
    }
    return W;
}

template <int P>
const void *window_kernel_p()
{
    constexpr Plan Q = kPlans[P];
    static_assert(!(Q.opt & 1024), "window mode: 8-wave workgroups");
    return plan_kernel<Q.G, Q.CH, Q.NBUF, Q.opt | kWinOpt>();
}

// the window kernel of W's plan: G = 64 for multiples of 4 KiB, G = 16 (four
// blocks per wave group) for the other whole KiB multiples
const void *window_fn(int p)
{
    switch (p) {
    case PLAN_4K: return window_kernel_p<PLAN_4K>();
    case PLAN_4K_DEEP: return window_kernel_p<PLAN_4K_DEEP>();
    case PLAN_G64_CH4_NIB: return window_kernel_p<PLAN_G64_CH4_NIB>();
    case PLAN_G16_CH4: return window_kernel_p<PLAN_G16_CH4>();
    case PLAN_G16_CH4_PIPE: return window_kernel_p<PLAN_G16_CH4_PIPE>();
    default: return window_kernel_p<PLAN_G64_CH4>();
    }
}

int launch_stride(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t *out,
                  hipStream_t s);

// the XCD weights of a window launch over nblocks (one launch: from 32
// groups per resident wave, as launch_plan applies them)
uint32_t window_xw(const priskv_crc_ctx *ctx, int p, uint64_t nblocks)
{
    const uint64_t n = nblocks / (64 / (uint64_t)kPlans[p].G), NW = (uint64_t)plan_waves(p);
    const uint64_t max_wgs = (uint64_t)ctx->num_cus * ctx->plan_wgs_per_cu[p];
    const uint64_t want = (n + NW - 1) / NW, grid = want < max_wgs ? want : max_wgs;
    return n >= 32ull * grid * NW ? ctx->plan_xw[p] : 0u;
}

int launch_window(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t W,
                  uint32_t *out, hipStream_t s)
{
    const int p = plan_for(W, nblocks);
    const Plan &P = kPlans[p];
    const uint64_t per = 64 / (uint64_t)P.G; // blocks per wave group
    const int gi = P.G == 64 ? 0 : (P.G == 32 ? 1 : 2);
    const uint64_t max_wgs = (uint64_t)ctx->num_cus * ctx->plan_wgs_per_cu[p];
    const uint64_t NW = (uint64_t)plan_waves(p);
    const uint64_t cps = W / ((uint64_t)P.CH * 16u * P.G);
    const uint32_t *img = ctx->d_lds_image[gi];
    const uint32_t *fold = (P.opt & 32) ? ctx->d_nibrep[log2u(P.G)] : ctx->d_fold + log2u(P.G) * 2048;
    const uint32_t *zp = ctx->d_winimg + (W / 1024 - 1) * kWinImgWords; // (s_winimg)
    const uint64_t cap = max_wgs * NW * ((1ull << 31) / cps - 1);
    const uint64_t ngroups = nblocks / per;
    for (uint64_t done = 0; done < ngroups;) {
        uint64_t n = (ngroups - done < cap) ? ngroups - done : cap;
        const uint64_t want = (n + NW - 1) / NW;
        const uint32_t grid = (uint32_t)(want < max_wgs ? want : max_wgs);
        const uint8_t *b = base + done * per * bs;
        uint32_t *o = out + done * per;
        uint32_t xw = n >= 32ull * grid * NW ? ctx->plan_xw[p] : 0u, tile = 0, one = 1, stride = bs, wb = W;
        uint64_t *none = nullptr;
        void *args[] = {(void *)&b,  (void *)&n,    (void *)&wb,   (void *)&img,    (void *)&fold,
                        (void *)&o,  (void *)&xw,   (void *)&tile, (void *)&stride, (void *)&one,
                        (void *)&zp, (void *)&none};
        if (int rc = herr(hipLaunchKernel(window_fn(p), dim3(grid), dim3(64 * NW), args, 0, s)))
            return rc;
        done += n;
    }
    // a ragged tail of fewer than a group's blocks (G = 16): the stride kernel
    // or, from 9 KiB, the extents kernel
    const uint64_t head = ngroups * per;
    if (head == nblocks)
        return 0;
    if (bs >= kStrideMax)
        return launch_extents(ctx, base + head * bs, nblocks - head, nullptr, nullptr, bs, bs, out + head, s);
    return launch_stride(ctx, base + head * bs, nblocks - head, bs, out + head, s);
}

// sub-KiB kernel for G = 1 << gl: no fold at G = 1 (a lane holds a whole
// block); G = 2-16 the byte-table fold, G = 32 the nibble fold; with prio in
// one 16-wave workgroup per CU and progress-priority mode 1 (+0.2-2.6 % at
// 32-512 B, profiles/r01/prio/small_*.log; round 3 +5 % at 16 B,
// profiles/r03/bytefold/), else in two 8-wave workgroups per CU
// (PRISKV_CRC_PRIO=0)
constexpr int kSmallOptPrio = 1 | (1 << 8) | 1024;

// Chunk shape: 4 rows per chunk with 3 chunks in the register pipeline
// (was 2): +1.3-2.8 % for G >= 2 and +2.2-2.8 % for G = 1, 1 GiB per call
// (profiles/r02/small/).  8 rows 3 deep was 1.5 % faster still at G = 1,
// but at 182 VGPRs it halves the resident waves.
constexpr int kSmallCh = 4, kSmallNbuf = 3, kSmallCh1 = 4, kSmallNbuf1 = 3;

// byte-table fold (OPT bit 1) for G = 2..16: four lookups per fold instead
// of eight nibble lookups (crc_device.inc byte_fold)
template <int G>
const void *small_fn_g()
{
    if constexpr (G <= 16) // first chunks before the tables (OPT bit 2): 256 MiB calls -2.5-3 %, 4 GiB level
        return reinterpret_cast<const void *>(&crc_small_kernel<G, kSmallOptPrio | 2 | 4, kSmallCh, kSmallNbuf>);
    return reinterpret_cast<const void *>(&crc_small_kernel<G, kSmallOptPrio, kSmallCh, kSmallNbuf>);
}

// G = 1 << gl lanes per block: G = 2..16 fold through the byte tables, G = 32
// through the nibble tables, G = 1 needs no fold; all in one 16-wave
// workgroup per CU with progress priority
const void *small_fn(int gl)
{
    switch (gl) {
    case 0: return reinterpret_cast<const void *>(&crc_small_kernel<1, kSmallOptPrio, kSmallCh1, kSmallNbuf1>);
    case 1: return small_fn_g<2>();
    case 2: return small_fn_g<4>();
    case 3: return small_fn_g<8>();
    case 4: return small_fn_g<16>();
    default: return small_fn_g<32>();
    }
}

// ---- uniform-stride kernel (odd block sizes, unaligned bases) ------------------
// G lanes per block with R = ceil(B / 16G) rows; G < 16 only for R = 1 (the
// set-B row jump exists for G = 16, 32, 64).  Score = the share of hashed
// bytes that are block bytes, B / (16G (R + 1/2)) (half a row for the fold),
// times 0.88 for G <= 16: runs of 256 B or less per block and row read
// slower from unaligned starts (tools/stride_sweep.py, profiles/r02/stride/:
// 4100 B G32 5.81 against G16 5.30 TB/s, 1500 B 5.58 / 5.31, 520 B G16
// 4.42 / G32 3.59).  4100 B -> G32 x 9 rows, 1000 B -> G32 x 2, 520 B ->
// G16 x 3, 100 B -> G8 x 1.
struct StridePlan {
    int G;
    uint32_t R;
};
// Odd block sizes or bases (not multiples of 4) and other sizes from 9 KiB
// take the extents kernel: its 16-B aligned windows and one fold per block
// beat the stride kernel's per-row work once a block spans 9-10 of its rows.
// Round 2 (profiles/r02/stride/, TB/s extents / stride): odd 4097 B 4.80 /
// 5.52, 16 385 B 6.32 / 5.19; multiples of 4 14 340 B 6.42 / 5.99.  Round 3,
// with progress priority in one 16-wave workgroup, the stride kernel leads
// odd sizes up to 8.5 KiB (4609 B 5.84 / 5.19 extents, 8193 B 6.10 / 5.70,
// 8705 B 6.01 / 5.88) and trails from 9 KiB (9217 B 6.04 / 6.11, 10 241 B
// 6.01 / 6.37; profiles/r03/stride_prio/).
bool stride_to_extents(const void *base, uint32_t bs)
{
    (void)base;
    return bs >= kStrideMax;
}

// the extents-path kernels a batch of n extents of at most max_len bytes
// launches (max_len 0: lengths on the device)
const char *extents_desc(const priskv_crc_ctx *ctx, uint64_t n, uint64_t max_len)
{
    if (!extents_segmented(ctx, n, max_len))
        return "crc_ranges_kernel (extents)";
    return ctx->fused ? "crc_ranges_fused_kernel (few large values: segments, one launch)"
                      : "crc_seg_plan_kernel + crc_ranges_kernel (segments) + crc_seg_reduce_kernel";
}

StridePlan stride_plan(uint32_t bs)
{
    StridePlan best{0, 0};
    double bsc = -1.0;
    for (int G = 2; G <= 32; G *= 2) {
        const uint32_t RB = 16u * (uint32_t)G, R = (uint32_t)(((uint64_t)bs + RB - 1) / RB);
        if (G < 16 && R > 1)
            continue;
        // rows used / rows loaded (half a row of front slack on average),
        // G <= 16 marked down.  (G = 64 never wins below the 9 KiB limit:
        // 4096 B at an unaligned base G32 0.94 against G64 0.89.)
        const double score = (double)bs / (RB * (R + 0.5)) * (G <= 16 ? 0.88 : 1.0);
        if (score > bsc) {
            bsc = score;
            best = {G, R};
        }
    }
    return best;
}

// Chunks of 8 rows, 2 in flight (4 x 3, 2 x 4 and 4 x 2 differed by 2-8 %
// either way with the context order and were dropped: profiles/r02/stride/
// sweep_tune.jsonl), one 16-wave workgroup per CU with progress-priority
// mode 3 (round 3: +7-10 % at 1000-6000 B over two 8-wave workgroups).
// odd: a block size or base that is not a multiple of 4 -- aligned loads and
// funnel shifts (unaligned loads stream at 5.3 of 7.0 TB/s).
// G <= 8 (R = 1, set B unused): the byte-table fold in the sub-KiB image.
// G >= 16 with aligned loads also requests its first chunks before the
// tables (256 MiB of 1000-B blocks -2-5 %; the funnel-shift variant lost 5 %
// at 4097 B and G <= 8 was level: profiles/r03/early/).
template <int G>
const void *stride_fn_g(bool odd)
{
    if constexpr (G >= 16)
        return odd ? reinterpret_cast<const void *>(&crc_stride_kernel<G, 8, 2, kAux, true, false, 3>)
                   : reinterpret_cast<const void *>(&crc_stride_kernel<G, 8, 2, kAux, false, false, 3, true>);
    else
        return odd ? reinterpret_cast<const void *>(&crc_stride_kernel<G, 8, 2, kAux, true, true, 3>)
                   : reinterpret_cast<const void *>(&crc_stride_kernel<G, 8, 2, kAux, false, true, 3>);
}

const void *stride_fn(int G, bool odd)
{
    switch (G) {
    case 2: return stride_fn_g<2>(odd);
    case 4: return stride_fn_g<4>(odd);
    case 8: return stride_fn_g<8>(odd);
    case 16: return stride_fn_g<16>(odd);
    default: return stride_fn_g<32>(odd);
    }
}

int launch_stride(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs, uint32_t *out,
                  hipStream_t s)
{
    const StridePlan P = stride_plan(bs);
    const uint64_t NB = 64 / (uint64_t)P.G;
    const bool bf = P.G <= 8;
    const uint64_t nw = 16;
    const uint64_t max_wgs = (uint64_t)ctx->num_cus;
    // a wave's range is one buffer descriptor with 31-bit offsets, and its
    // NB lane groups may run up to NB - 1 blocks past it: cap blocks per launch
    const uint64_t per_wave = ((1ull << 31) - 1) / bs - NB; // >= 1: bs < kStrideMax
    const uint64_t cap = max_wgs * nw * per_wave;
    const uint32_t *img = bf ? ctx->d_small_img[log2u((uint32_t)P.G)]
                             : ctx->d_lds_image[P.G == 32 ? 1 : 2]; // set B unused for G < 16
    const uint32_t *nib = ctx->d_nibrep[log2u((uint32_t)P.G)];
    uint32_t R = P.R;
    for (uint64_t done = 0; done < nblocks;) {
        uint64_t nb = nblocks - done < cap ? nblocks - done : cap;
        const uint64_t want = (nb + NB * nw - 1) / (NB * nw); // about NB blocks per wave and up
        const uint32_t grid = (uint32_t)(want < max_wgs ? want : max_wgs);
        const uint8_t *b = base + done * bs;
        const void *fn = stride_fn(P.G, (((uintptr_t)b | bs) & 3u) != 0);
        uint32_t *o = out + done;
        void *args[] = {(void *)&b, (void *)&nb, (void *)&bs, (void *)&R, (void *)&img, (void *)&nib, (void *)&o};
        if (int rc = herr(hipLaunchKernel(fn, dim3(grid), dim3(64 * nw), args, 0, s)))
            return rc;
        done += nb;
    }
    return 0;
}

int launch_blocks(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs,
                  uint32_t *out, hipStream_t s)
{
    const int path = choose_path(base, bs);
    if (path == PATH_ROWS)
        return launch_rows(ctx, base, nblocks, bs, out, s);
    // the window mode before the head split: level or faster wherever both
    // apply (profiles/r05/window/headsplit_vs_window.jsonl: 1064 B +13 %,
    // 2056 / 3080 B +3-4 %, 4104 / 4144 B +2 %, 1040 B level)
    if (path == PATH_STRIDE)
        if (const uint32_t W = window_bytes(ctx, base, nblocks, bs))
            return launch_window(ctx, base, nblocks, bs, W, out, s);
    if (path == PATH_STRIDE && head_split(ctx, base, nblocks, bs))
        return launch_head_split(ctx, base, nblocks, bs, out, s);
    if (path == PATH_STRIDE && !stride_to_extents(base, bs))
        return launch_stride(ctx, base, nblocks, bs, out, s);
    if (path == PATH_STRIDE) // from 9 KiB: extents (segmented when few)
        return launch_extents(ctx, base, nblocks, nullptr, nullptr, bs, bs, out, s);
    if (path == PATH_SMALL) {
        const int gl = log2u(bs / 16); // G = 1 << gl
        const uint64_t per = 1024 / bs; // blocks per row
        const uint64_t nrows = nblocks / per;
        if (nrows) {
            // G = 2..16: byte-table fold (the sub-KiB images), G = 32: nibble-table
            // fold (replicated 32-wide tables); one 16-wave workgroup per CU
            const bool bf = gl >= 1 && gl <= 4;
            const uint32_t *fold = gl ? ctx->d_nibrep[gl] : ctx->d_fold;
            const uint32_t *img = bf ? ctx->d_small_img[gl] : ctx->d_lds_image[0];
            const int waves = 2 * kWaves;
            const uint64_t cap = (uint64_t)ctx->num_cus;
            const uint64_t chw = (uint64_t)(gl == 0 ? kSmallCh1 : kSmallCh) * waves; // rows per wave-chunk
            const uint64_t want = (nrows + chw - 1) / chw;
            const uint32_t grid = (uint32_t)(want < cap ? want : cap);
            void *args[] = {(void *)&base, (void *)&nrows, (void *)&img, (void *)&fold, (void *)&out};
            if (int rc = herr(hipLaunchKernel(small_fn(gl), dim3(grid), dim3(64 * waves), args, 0, s)))
                return rc;
        }
        const uint64_t head = nrows * per;
        if (head == nblocks)
            return 0;
        return launch_generic(ctx, base + head * bs, nblocks - head, bs, bs, nullptr, nullptr, out + head, s);
    }
    if (bs >= PRV_ROW_BYTES)
        return launch_extents(ctx, base, nblocks, nullptr, nullptr, bs, bs, out, s);
    return launch_generic(ctx, base, nblocks, bs, bs, nullptr, nullptr, out, s);
}

// XCD weights of the rows-kernel split: on a multi-XCD device
// (workgroups dispatched round-robin over 8 XCDs) waves on odd XCDs finish
// later under an equal split on every MI355X measured, so even-XCD waves take
// more parts (kPlans[p].we : wo).  Only when the context's probe saw
// workgroup b on XCD (b + k) % 8 (xcd_rr); otherwise -- another partition mode, a
// different XCD count -- the split is equal.  PRISKV_CRC_XCD_WEIGHTS="we:wo"
// overrides every plan ("1:1" = equal split) and applies regardless.
uint32_t xcd_weights(int xcd_rr, int p)
{
    // no round-robin dispatch found (another partition mode, the probe off):
    // equal shares whatever the environment says -- the kernels' per-workgroup
    // weight order (wave_range) is consistent across a launch only under
    // round-robin dispatch
    if (!xcd_rr)
        return 0u;
    uint32_t we = kPlans[p].we, wo = kPlans[p].wo;
    if (const char *e = getenv("PRISKV_CRC_XCD_WEIGHTS")) {
        unsigned a = 0, b = 0;
        if (sscanf(e, "%u:%u", &a, &b) == 2 && a && b && a < 65536 && b < 65536) {
            we = a;
            wo = b;
        }
    }
    return we == wo ? 0u : ((we << 16) | wo);
}

// Does workgroup b of a launch run on XCD (b + k) % 8 (8 XCDs, round-robin
// from some first XCD k)?
// One launch of 64 single-wave workgroups on the context's stream.
// PRISKV_CRC_XCD_PROBE=0 forces "no" (tests of the fallback).
int xcd_probe(priskv_crc_ctx *c, int *rr)
{
    *rr = 0;
    if (const char *e = getenv("PRISKV_CRC_XCD_PROBE"))
        if (!strcmp(e, "0"))
            return 0;
    if (c->num_cus < 64 || c->num_cus % 8)
        return 0;
    constexpr int kProbeWgs = 64;
    uint32_t *d = nullptr;
    uint32_t h[kProbeWgs];
    int rc = herr(hipMalloc((void **)&d, sizeof(h)));
    if (rc)
        return rc;
    if (!(rc = launch_k(crc_xcd_probe_kernel, dim3(kProbeWgs), dim3(64), c->aux, d)) &&
        !(rc = herr(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->aux))))
        rc = herr(hipStreamSynchronize(c->aux));
    (void)hipFree(d);
    if (rc)
        return rc;
    // round-robin from the queue's first XCD (which differs by hardware queue:
    // the kernels read its parity themselves, wave_range)
    int ok = h[0] < 8;
    for (int b = 0; b < kProbeWgs; b++)
        ok &= h[b] == (h[0] + (uint32_t)b) % 8;
    *rr = ok;
    return 0;
}

// resident workgroups per CU of every plan: the plan's choice, capped by
// what the runtime can actually co-schedule (VGPR / LDS limits)
int rows_occupancy(priskv_crc_ctx *c)
{
    for (int p = 0; p < NPLANS; p++) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, plan_fn(p), 64 * plan_waves(p), 0);
        if (e != hipSuccess)
            return herr(e);
        c->plan_wgs_per_cu[p] = n < 1 ? 1 : (n < kPlans[p].wg_per_cu ? n : kPlans[p].wg_per_cu);
    }
    return 0;
}

} // namespace

extern "C" {

const char *priskv_crc_version(void) { return PRV_VERSION; }

int priskv_crc32_blocks_path(const void *d_base, uint64_t nblocks, uint32_t block_size)
{
    if (block_size == 0 || (nblocks && !d_base))
        return -EINVAL;
    const int path = choose_path(d_base, block_size);
    // a default context hashes B = h + whole KiB rows as bodies + heads
    // (unless few large blocks), and sends stride sizes from 9 KiB to the
    // extents kernel
    if (path == PATH_STRIDE && window_bytes(nullptr, d_base, nblocks, block_size))
        return PATH_WINDOW;
    if (path == PATH_STRIDE && head_split(nullptr, d_base, nblocks, block_size))
        return PATH_HEAD;
    if (path == PATH_STRIDE && stride_to_extents(d_base, block_size))
        return PATH_EXTENTS;
    return path;
}

int priskv_crc32_blocks_plan(const priskv_crc_ctx *ctx, const void *d_base, uint64_t nblocks, uint32_t block_size,
                             char *buf, uint64_t len)
{
    if (!ctx || block_size == 0 || !buf || len == 0)
        return -EINVAL;
    int path = choose_path(d_base, block_size);
    const uint32_t win = path == PATH_STRIDE ? window_bytes(ctx, d_base, nblocks, block_size) : 0u;
    if (!win && path == PATH_STRIDE && head_split(ctx, d_base, nblocks, block_size))
        path = PATH_HEAD;
    int w = 0;
    const char *fused_name = "crc_ranges_fused_kernel (few large values: segments, one launch)";
    if (win) {
        const int p = plan_for(win, nblocks);
        const Plan &P = kPlans[p];
        const uint32_t xw = window_xw(ctx, p, nblocks);
        char xs[32] = "";
        if (xw)
            snprintf(xs, sizeof(xs), ",xcd-weighted %u:%u", xw >> 16, xw & 0xFFFF);
        w = snprintf(buf, len,
                     "crc_rows_kernel<G=%d,CH=%d,NBUF=%d,nt%s%s,progress-priority %d,window%s> (%u-B windows ending "
                     "at the 16-B boundary after each block, corrected as each 64 CRCs are stored)",
                     P.G, P.CH, P.NBUF, (P.opt & 2) ? ",pipelined-fold" : "", (P.opt & 32) ? ",nibble-fold" : "",
                     (P.opt >> 8) & 3, xs, win);
    } else if (path == PATH_STRIDE) {
        const StridePlan P = stride_plan(block_size);
        if (stride_to_extents(d_base, block_size)) {
            w = snprintf(buf, len, "%s", extents_desc(ctx, nblocks, block_size));
        } else {
            const int ch = 8, nbuf = 2;
            w = snprintf(buf, len,
                         "crc_stride_kernel<G=%d,CH=%d,NBUF=%d,nt%s,progress-priority 3> (%u rows of %u B per block, "
                         "%u B in front)",
                         P.G, ch, nbuf, P.G <= 8 ? ",byte-fold" : "", P.R, 16u * P.G, P.R * 16u * P.G - block_size);
        }
    } else if (path == PATH_ROWS && segments_for(ctx, nblocks, block_size) > 1 &&
               split_few(ctx, nblocks, block_size) > 1) {
        const uint32_t sf = split_few(ctx, nblocks, block_size);
        const uint32_t xw = split_units_xw(ctx, PLAN_SPLIT_DEEP, nblocks * sf);
        w = snprintf(buf, len,
                     "crc_rows_kernel<G=64,CH=4,NBUF=3,nt,nibble-fold%s,first chunks before the tables,"
                     "split %u units of %u B per block%s",
                     ",progress-priority 3", sf, block_size / sf, xw ? ",xcd-weighted" : "");
        if (w >= 0 && (uint64_t)w < len && xw)
            w += snprintf(buf + w, len - w, " %u:%u", xw >> 16, xw & 0xFFFF);
        if (w >= 0 && (uint64_t)w < len)
            w += snprintf(buf + w, len - w, "> (few large blocks)");
    } else if (path == PATH_ROWS && segments_for(ctx, nblocks, block_size) > 1 && fused_blocks(ctx, nblocks)) {
        w = snprintf(buf, len, "%s", fused_name);
    } else if (path == PATH_ROWS || path == PATH_HEAD) {
        const uint32_t hb = path == PATH_HEAD ? block_size % PRV_ROW_BYTES : 0u; // head bytes
        block_size -= hb;
        const uint32_t S = segments_for(ctx, nblocks, block_size);
        const uint32_t bs = block_size / S;
        const int p = plan_for(bs, nblocks * S);
        const Plan &P = kPlans[p];
        const uint32_t xw = ctx->plan_xw[p];
        const int mode = (P.opt >> 8) & 3;
        w = snprintf(buf, len, "crc_rows_kernel<G=%d,CH=%d,NBUF=%d,nt%s%s", P.G, P.CH, P.NBUF,
                     (P.opt & 2) ? ",pipelined-fold" : "", (P.opt & 32) ? ",nibble-fold" : "");
        if (w >= 0 && (uint64_t)w < len && mode)
            w += snprintf(buf + w, len - w, ",progress-priority %d", mode);
        const uint64_t ngroups = nblocks * S / (64 / P.G);
        const uint32_t tile = tile_groups(ctx, ngroups, (uint64_t)(64 / P.G) * bs);
        const uint32_t sp = (S == 1 && !hb) ? split_for(ctx, nblocks, bs) : 1u;
        if (w >= 0 && (uint64_t)w < len && sp > 1)
            w += snprintf(buf + w, len - w, ",split %u units of %u B per block,xcd-weighted %u:%u", sp, bs / sp,
                          xw >> 16, xw & 0xFFFF);
        else if (w >= 0 && (uint64_t)w < len && tile)
            w += snprintf(buf + w, len - w, ",block-cyclic tiles of %u groups", tile);
        else if (w >= 0 && (uint64_t)w < len && xw && ngroups >= 32ull * ctx->num_cus * ctx->plan_wgs_per_cu[p] * kWaves)
            w += snprintf(buf + w, len - w, ",xcd-weighted %u:%u", xw >> 16, xw & 0xFFFF);
        if (w >= 0 && (uint64_t)w < len)
            w += snprintf(buf + w, len - w, ">%s", S > 1 ? " x segments + crc_combine_segments_kernel" : "");
        if (w >= 0 && (uint64_t)w < len && S > 1)
            w += snprintf(buf + w, len - w, " (%u segments of %u B per block)", S, bs);
        if (w >= 0 && (uint64_t)w < len && hb)
            w += snprintf(buf + w, len - w, " on the %u-B bodies + crc_head_kernel (%u-B heads)", block_size, hb);
    } else if (path == PATH_SMALL) {
        const uint32_t G = block_size / 16;
        w = snprintf(buf, len, "crc_small_kernel<G=%u%s>", G, (G >= 2 && G <= 16) ? ",byte-fold" : "");
    } else if (path == PATH_EXTENTS) {
        w = snprintf(buf, len, "%s", extents_desc(ctx, nblocks, block_size));
    } else {
        w = snprintf(buf, len, "crc_generic_kernel");
    }
    return w < 0 ? -EIO : 0;
}

int priskv_crc_read_roof_dev(const priskv_crc_ctx *ctx, const void *d_base, uint64_t nblocks, uint32_t block_size,
                             uint32_t variant, uint32_t *d_sink, void *stream)
{
    if (!ctx || block_size == 0 || ((uintptr_t)d_base & 15) != 0 || variant >= PRISKV_CRC_ROOF_VARIANTS)
        return -EINVAL;
    // an odd block size the window mode takes with a 4 KiB-multiple window:
    // the roof reads the windows (crc_read_roof_kernel stride)
    uint32_t stride = 0;
    if (block_size % 4096 != 0) {
        const uint32_t W = window_bytes(ctx, d_base, nblocks, block_size);
        if (!W || W % 4096 != 0)
            return -EINVAL;
        stride = block_size;
        block_size = W;
    }
    if (nblocks == 0)
        return 0;
    if (!d_base || !d_sink)
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    // the plan the CRC kernel uses for this block size: its resident
    // workgroups and pipeline depth (variant 0; variants 1-6: NBUF 2 / 3 / 4
    // at one or two 8-wave workgroups per CU), its split mode (units of
    // block_size / S) and its XCD weights (only with many units per wave, as
    // launch_plan applies them); the roof reads units as blocks
    int p = plan_for(block_size, nblocks);
    uint32_t S = 1;
    if (stride) // (launch_window: the W plan, whole blocks, no tiles)
        ;
    else if (segments_for(ctx, nblocks, block_size) == 1)
        S = split_for(ctx, nblocks, block_size);
    else if ((S = split_few(ctx, nblocks, block_size)) > 1)
        p = PLAN_SPLIT_DEEP;
    // variants 7-8: the plan's shape with progress priority mode 1 / 3
    const int nbuf = (variant && variant < 7) ? 2 + (int)(variant - 1) / 2 : kPlans[p].NBUF;
    const uint64_t wgpc = (variant && variant < 7) ? 1 + (variant - 1) % 2 : (uint64_t)ctx->plan_wgs_per_cu[p];
    const int prio = variant == 7 ? 1 : variant == 8 ? 3 : 0;
    const uint64_t max_wgs = (uint64_t)ctx->num_cus * wgpc;
    block_size /= S;
    nblocks *= S;
    const uint64_t cps = block_size / 4096;
    const uint64_t want = (nblocks + kWaves - 1) / kWaves;
    const uint32_t grid = (uint32_t)(want < max_wgs ? want : max_wgs);
    // one launch (a wave's chunk count is 32-bit) and one sink slot per wave
    if ((uint64_t)grid * kWaves > PRISKV_CRC_ROOF_SINK_WORDS || (nblocks + grid * kWaves - 1) / (grid * kWaves) * cps >= (1ull << 31))
        return -EINVAL;
    const uint8_t *b = static_cast<const uint8_t *>(d_base);
    uint32_t bs = block_size;
    uint32_t xw = nblocks >= 32ull * grid * kWaves ? ctx->plan_xw[p] : 0u;
    uint32_t tile = S == 1 && !stride ? tile_groups(ctx, nblocks, bs) : 0u; // the CRC kernel's tiles (G = 64: a group is a block)
    if (tile)
        xw = 0;
    const void *fn = nbuf == 4   ? (prio == 1   ? reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 4, kAux, 1>)
                                    : prio == 3 ? reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 4, kAux, 3>)
                                                : reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 4, kAux>))
                     : nbuf == 3 ? (prio == 1   ? reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 3, kAux, 1>)
                                    : prio == 3 ? reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 3, kAux, 3>)
                                                : reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 3, kAux>))
                                 : (prio == 1   ? reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 2, kAux, 1>)
                                    : prio == 3 ? reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 2, kAux, 3>)
                                                : reinterpret_cast<const void *>(&crc_read_roof_kernel<4, 2, kAux>));
    void *args[] = {(void *)&b, (void *)&nblocks, (void *)&bs, (void *)&d_sink, (void *)&xw, (void *)&tile,
                    (void *)&stride};
    return herr(hipLaunchKernel(fn, dim3(grid), dim3(kThreads), args, 0, (hipStream_t)stream));
}

int priskv_crc_ctx_create(int device, priskv_crc_ctx **out)
{
    if (!out)
        return -EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev)
        return -ENODEV;
    DevGuard g(device);
    if (!g.ok)
        return -ENODEV;
    priskv_crc_ctx *c = (priskv_crc_ctx *)calloc(1, sizeof(*c));
    if (!c)
        return -ENOMEM;
    c->device = device;
    pthread_mutex_init(&c->lock, NULL);
    pthread_mutex_init(&c->pool_lock, NULL);
    int rc = 0;
    uint32_t *h_img = (uint32_t *)malloc(sizeof(uint32_t) * PRV_LDS_WORDS);
    uint32_t *h_fold = (uint32_t *)malloc(sizeof(uint32_t) * 2048 * kFoldSets);
    uint32_t h_sar[256];
    static_assert(16 * 4 * 32 <= PRV_LDS_WORDS, "rowshift image fits the staging buffer");
    if (!h_img || !h_fold) {
        rc = -ENOMEM;
        goto fail;
    }
    if ((rc = herr(hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, device))))
        goto fail;
    {
        const char *e = getenv("PRISKV_CRC_SEGMENT");
        c->segment = !(e && !strcmp(e, "0"));
        const char *sp = getenv("PRISKV_CRC_SPLIT");
        c->split = !(sp && !strcmp(sp, "0"));
        const char *be = getenv("PRISKV_CRC_BALANCE");
        c->balance = !(be && !strcmp(be, "0"));
        const char *hs = getenv("PRISKV_CRC_HEADSPLIT");
        c->head_split = !(hs && !strcmp(hs, "0"));
        const char *we = getenv("PRISKV_CRC_WINDOW");
        c->window = !(we && !strcmp(we, "0"));
        const char *fe = getenv("PRISKV_CRC_FUSED");
        c->fused = !(fe && !strcmp(fe, "0"));
        c->seg_max_extents = kSegMaxExtents;
        c->tile_min_bytes = kTileMinBytes;
        c->tile_bytes = kTileBytes;
        if (const char *m = getenv("PRISKV_CRC_TILE_MIN_GIB"))
            c->tile_min_bytes = strtoull(m, nullptr, 10) << 30;
        if (const char *m = getenv("PRISKV_CRC_TILE_KIB")) {
            const unsigned long long v = strtoull(m, nullptr, 10);
            c->tile_bytes = v ? v << 10 : kTileBytes;
        }
        if (const char *m = getenv("PRISKV_CRC_SEG_MAX_EXTENTS")) { // capped by the plan kernel's 16384
            const unsigned long long v = strtoull(m, nullptr, 10);
            const uint64_t cap = (uint64_t)kSegPlanThreads * kSegPlanPerThread;
            c->seg_max_extents = v < cap ? v : cap;
        }
    }
    for (int j = 0; j < kFoldSets; j++)
        prv_fold_columns(h_fold + j * 2048, 1u << j);
    prv_sarwate_table(h_sar);
    if ((rc = herr(hipMalloc((void **)&c->d_fold, sizeof(uint32_t) * 2048 * kFoldSets))) ||
        (rc = herr(hipMalloc((void **)&c->d_sarwate, sizeof(h_sar)))) ||
        (rc = herr(hipMalloc((void **)&c->d_rowshift, sizeof(uint32_t) * 16 * 4 * 32))) ||
        (rc = herr(hipMalloc((void **)&c->d_zpow, sizeof(uint32_t) * kZpowRows * 32))))
        goto fail;
    if ((rc = herr(hipMemcpy(c->d_fold, h_fold, sizeof(uint32_t) * 2048 * kFoldSets, hipMemcpyHostToDevice))) ||
        (rc = herr(hipMemcpy(c->d_sarwate, h_sar, sizeof(h_sar), hipMemcpyHostToDevice))))
        goto fail;
    prv_rowshift_columns(h_img);
    if ((rc = herr(hipMemcpy(c->d_rowshift, h_img, sizeof(uint32_t) * 16 * 4 * 32, hipMemcpyHostToDevice))))
        goto fail;
    if ((rc = herr(hipMalloc((void **)&c->d_winimg, sizeof(uint32_t) * kWinImages * kWinImgWords))))
        goto fail;
    static_assert(kWinImgWords <= PRV_LDS_WORDS, "a window image fits the staging buffer");
    for (int wi = 0; wi < kWinImages; wi++) {
        uint32_t *im = h_img;
        const uint32_t W = 1024u * (uint32_t)(wi + 1);
        prv_sarwate_table(im);
        for (int k = 1; k < 4; k++)
            for (int i = 0; i < 256; i++) {
                const uint32_t v = im[(k - 1) * 256 + i];
                im[k * 256 + i] = (v >> 8) ^ im[v & 0xff];
            }
        // nibble tables: Z_W, Z_(W - 16), Z_-p (p = 0..15)
        uint32_t cols[18][32];
        prv_shift_columns(cols[0], W);
        prv_shift_columns(cols[1], W - 16);
        prv_unshift_columns(&cols[2][0]);
        for (int t = 0; t < 18; t++)
            for (int nb = 0; nb < 8; nb++)
                for (uint32_t v = 0; v < 16; v++) {
                    uint32_t r = 0;
                    for (int bit = 0; bit < 4; bit++)
                        if ((v >> bit) & 1u)
                            r ^= cols[t][4 * nb + bit];
                    im[4 * 256 + t * kWinNib + nb * 16 + (int)v] = r;
                }
        if ((rc = herr(hipMemcpy(c->d_winimg + wi * kWinImgWords, h_img, sizeof(uint32_t) * kWinImgWords,
                                 hipMemcpyHostToDevice))))
            goto fail;
    }
    for (int k = 0; k < kZpowRows; k++)
        prv_shift_columns(h_img + k * 32, 1ull << k);
    if ((rc = herr(hipMemcpy(c->d_zpow, h_img, sizeof(uint32_t) * kZpowRows * 32, hipMemcpyHostToDevice))))
        goto fail;
    for (int gi = 0; gi < 3; gi++) {
        const uint32_t G = 64u >> gi; // 64, 32, 16
        prv_lds_image(h_img, 16u * G - 16u);
        if ((rc = herr(hipMalloc((void **)&c->d_lds_image[gi], sizeof(uint32_t) * PRV_LDS_WORDS))) ||
            (rc = herr(hipMemcpy(c->d_lds_image[gi], h_img, sizeof(uint32_t) * PRV_LDS_WORDS, hipMemcpyHostToDevice))))
            goto fail;
    }
    for (int j = 1; j < kFoldSets; j++) {
        const uint32_t G = 1u << j, W = G > 32 ? G : 32;
        prv_fold_nibbles(h_img, G, W); // 8 x 16 x W words fit in the image buffer
        if ((rc = herr(hipMalloc((void **)&c->d_nibrep[j], sizeof(uint32_t) * 8 * 16 * W))) ||
            (rc = herr(hipMemcpy(c->d_nibrep[j], h_img, sizeof(uint32_t) * 8 * 16 * W, hipMemcpyHostToDevice))))
            goto fail;
    }
    for (int j = 1; j <= 4; j++) {
        const uint32_t G = 1u << j;
        std::vector<uint32_t> simg(PRV_SMALL_WORDS(G));
        prv_small_image(simg.data(), G);
        if ((rc = herr(hipMalloc((void **)&c->d_small_img[j], sizeof(uint32_t) * simg.size()))) ||
            (rc = herr(hipMemcpy(c->d_small_img[j], simg.data(), sizeof(uint32_t) * simg.size(),
                                 hipMemcpyHostToDevice))))
            goto fail;
    }
    prv_fold_nibbles(h_img, 16, 16);
    if ((rc = herr(hipMalloc((void **)&c->d_nib16, sizeof(uint32_t) * 8 * 16 * 16))) ||
        (rc = herr(hipMemcpy(c->d_nib16, h_img, sizeof(uint32_t) * 8 * 16 * 16, hipMemcpyHostToDevice))))
        goto fail;
    if ((rc = rows_occupancy(c)))
        goto fail;
    if ((rc = herr(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking))))
        goto fail;
    if ((rc = xcd_probe(c, &c->xcd_rr)))
        goto fail;
    for (int p = 0; p < NPLANS; p++)
        c->plan_xw[p] = xcd_weights(c->xcd_rr, p);
    {
        const char *pe = getenv("PRISKV_CRC_SCRATCH_POOL");
        c->pool_ready = !(pe && !strcmp(pe, "0"));
    }
    free(h_img);
    free(h_fold);
    *out = c;
    return 0;
fail:
    free(h_img);
    free(h_fold);
    priskv_crc_ctx_destroy(c);
    return rc;
}

void priskv_crc_ctx_destroy(priskv_crc_ctx *c)
{
    if (!c)
        return;
    DevGuard g(c->device);
    free_deferred(true);
    if (c->stream_ready) {
        for (int i = 0; i < NSTREAM; i++) {
            (void)hipStreamSynchronize(c->streams[i]);
            (void)hipStreamDestroy(c->streams[i]);
            (void)hipFree(c->d_stage[i]);
            (void)hipFree(c->d_stage_out[i]);
            (void)hipHostFree(c->h_bounce[i]);
            (void)hipHostFree(c->h_out_stage[i]);
        }
    }
    for (int gi = 0; gi < 3; gi++)
        (void)hipFree(c->d_lds_image[gi]);
    for (int j = 0; j < kFoldSets; j++)
        (void)hipFree(c->d_nibrep[j]);
    (void)hipFree(c->d_nib16);
    for (int j = 1; j <= 4; j++)
        (void)hipFree(c->d_small_img[j]);
    (void)hipFree(c->d_fold);
    (void)hipFree(c->d_sarwate);
    (void)hipFree(c->d_rowshift);
    (void)hipFree(c->d_winimg);
    (void)hipFree(c->d_zpow);
    (void)hipFree(c->d_scrub);
    {
        // the slots' last uses are on their home streams, which may be gone
        // by now: wait for the device before freeing them
        bool any = false;
        for (priskv_crc_pool_slot *slots : {c->pool, c->cnt_pool})
            for (int i = 0; i < NPOOL; i++)
                any = any || slots[i].p;
        if (any)
            (void)hipDeviceSynchronize();
        for (priskv_crc_pool_slot *slots : {c->pool, c->cnt_pool})
            for (int i = 0; i < NPOOL; i++) {
                if (slots[i].p && slots[i].plain)
                    (void)hipFree(slots[i].p);
                else if (slots[i].p)
                    (void)hipFreeAsync(slots[i].p, c->aux);
                if (slots[i].ev)
                    (void)hipEventDestroy(slots[i].ev);
            }
    }
    if (c->aux) {
        (void)hipStreamSynchronize(c->aux);
        (void)hipStreamDestroy(c->aux);
    }
    pthread_mutex_destroy(&c->pool_lock);
    pthread_mutex_destroy(&c->lock);
    free(c);
}

int priskv_crc_ctx_device(const priskv_crc_ctx *ctx) { return ctx ? ctx->device : -EINVAL; }

#ifdef PRISKV_CRC_COVERAGE
// test-only build (make cov, tests/test_gpu_graphs_pool.py): after the device
// is idle, out[0] = the groups the waves' ranges (wave_range) covered since the
// last take, out[1] = the sum of their indices; then zero both.  Not declared
// in include/ and absent from the product library.
extern "C" __attribute__((visibility("default"))) int priskv_crc_cov_take(const priskv_crc_ctx *ctx, uint64_t *out)
{
    if (!ctx || !out)
        return -EINVAL;
    DevGuard g(ctx->device);
    unsigned long long h[2] = {0, 0};
    if (int rc = herr(hipDeviceSynchronize()))
        return rc;
    if (int rc = herr(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cov), sizeof(h))))
        return rc;
    const unsigned long long z[2] = {0, 0};
    if (int rc = herr(hipMemcpyToSymbol(HIP_SYMBOL(g_cov), z, sizeof(z))))
        return rc;
    out[0] = h[0];
    out[1] = h[1];
    return 0;
}

// test-only build: the per-wave timing records of the last rows-kernel
// launches (g_wave_t: n <= 8192 records of 4 words), after the device is idle
extern "C" __attribute__((visibility("default"))) int priskv_crc_cov_waves(const priskv_crc_ctx *ctx, uint64_t *out,
                                                                          uint64_t n)
{
    if (!ctx || !out || n > (uint64_t)kCovWaves)
        return -EINVAL;
    DevGuard g(ctx->device);
    if (int rc = herr(hipDeviceSynchronize()))
        return rc;
    return herr(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), n * 4 * sizeof(uint64_t)));
}

// test-only build: the scratch pool's pooled takes, misses (no free slot of
// the stream or unowned) and takeovers (a completed armed slot of another
// stream) since the context was created
extern "C" __attribute__((visibility("default"))) int priskv_crc_cov_pool(const priskv_crc_ctx *ctx, uint64_t *out)
{
    if (!ctx || !out)
        return -EINVAL;
    pthread_mutex_lock(&ctx->pool_lock);
    out[0] = ctx->pool_calls;
    out[1] = ctx->pool_misses;
    out[2] = ctx->pool_takeovers;
    pthread_mutex_unlock(&ctx->pool_lock);
    return 0;
}
#endif

int priskv_crc_stream_release(const priskv_crc_ctx *ctx, void *stream)
{
    if (!ctx)
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    const hipStream_t s = (hipStream_t)stream;
    StreamKey key;
    {
        RelaxedCapture relaxed;
        if (int rc = herr(hipStreamSynchronize(s))) // the slots' last uses
            return rc;
        if (!stream_key(s, &key))
            return -EIO;
        free_deferred(true);
    }
    pthread_mutex_lock(&ctx->pool_lock);
    for (priskv_crc_pool_slot *slots : {ctx->pool, ctx->cnt_pool})
        for (int i = 0; i < NPOOL; i++) {
            priskv_crc_pool_slot &q = slots[i];
            if (!q.busy && slot_owned_by(q, key)) {
                q.homed = 0;
                q.armed = 0;
            }
        }
    pthread_mutex_unlock(&ctx->pool_lock);
    return 0;
}

int priskv_crc32_blocks_dev(const priskv_crc_ctx *ctx, const void *d_base, uint64_t nblocks,
                            uint32_t block_size, uint32_t *d_out, void *stream)
{
    if (!ctx || block_size == 0)
        return -EINVAL;
    if (nblocks == 0)
        return 0;
    if (!d_base || !d_out)
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    return launch_blocks(ctx, (const uint8_t *)d_base, nblocks, block_size, d_out, (hipStream_t)stream);
}

namespace {
int ranges_dev(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
               uint64_t n, uint32_t *d_out, hipStream_t stream, uint64_t max_len)
{
    if (!ctx)
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!d_base || !d_offsets || !d_lengths || !d_out)
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    return launch_extents(ctx, (const uint8_t *)d_base, n, d_offsets, d_lengths, 0, 0, d_out, stream, max_len);
}
} // namespace

int priskv_crc32_ranges_dev(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                            const uint32_t *d_lengths, uint64_t n, uint32_t *d_out, void *stream)
{
    return ranges_dev(ctx, d_base, d_offsets, d_lengths, n, d_out, (hipStream_t)stream, 0);
}

// max_len only steers launch_extents' choice of kernel (every path hashes
// any lengths exactly); lengths are u32, so larger bounds say nothing more
int priskv_crc32_ranges_dev_bounded(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                                    const uint32_t *d_lengths, uint64_t n, uint64_t max_len, uint32_t *d_out,
                                    void *stream)
{
    return ranges_dev(ctx, d_base, d_offsets, d_lengths, n, d_out, (hipStream_t)stream,
                      max_len < 0xFFFFFFFFull ? max_len : 0xFFFFFFFFull);
}

namespace {
int verify_dev(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
               uint64_t n, const uint32_t *d_expected, uint64_t *d_status, void *stream, uint64_t max_len)
{
    if (!ctx || !d_status)
        return -EINVAL;
    if (n && (!d_base || !d_offsets || !d_lengths || !d_expected))
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    hipStream_t s = (hipStream_t)stream;
    // status first: a zero-length verify still reports {0, UINT64_MAX}
    if (int rc = launch_k(crc_status_init_kernel, dim3(1), dim3(64), s, (unsigned long long *)d_status))
        return rc;
    if (n == 0)
        return 0;
    Scratch sc(ctx, s); // pooled, ordered by events: concurrent calls never share a slot
    if (int rc = sc.get(n * sizeof(uint32_t)))
        return rc;
    uint32_t *got = static_cast<uint32_t *>(sc.p);
    int rc = launch_extents(ctx, (const uint8_t *)d_base, n, d_offsets, d_lengths, 0, 0, got, s, max_len);
    if (!rc) {
        const uint64_t want = (n + 255) / 256;
        const uint32_t grid = (uint32_t)(want < (uint64_t)ctx->num_cus * 4 ? want : (uint64_t)ctx->num_cus * 4);
        rc = launch_k(crc_verify_kernel, dim3(grid), dim3(256), s, got, d_expected, n, (unsigned long long *)d_status);
    }
    const int frc = sc.release();
    return rc ? rc : frc;
}
} // namespace

int priskv_crc32_verify_dev(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                            const uint32_t *d_lengths, uint64_t n, const uint32_t *d_expected,
                            uint64_t *d_status, void *stream)
{
    return verify_dev(ctx, d_base, d_offsets, d_lengths, n, d_expected, d_status, stream, 0);
}

// max_len: a launch hint only, as priskv_crc32_ranges_dev_bounded's
int priskv_crc32_verify_dev_bounded(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                                    const uint32_t *d_lengths, uint64_t n, uint64_t max_len,
                                    const uint32_t *d_expected, uint64_t *d_status, void *stream)
{
    return verify_dev(ctx, d_base, d_offsets, d_lengths, n, d_expected, d_status, stream,
                      max_len < 0xFFFFFFFFull ? max_len : 0xFFFFFFFFull);
}

int priskv_crc_fill_splitmix_dev(const priskv_crc_ctx *ctx, void *d_dst, uint64_t nbytes, uint64_t seed,
                                 uint64_t word_offset, void *stream)
{
    if (!ctx)
        return -EINVAL;
    if (nbytes == 0)
        return 0;
    if (!d_dst || ((uintptr_t)d_dst & 15))
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    uint64_t want = (nbytes / 16 + 255) / 256;
    uint64_t cap = (uint64_t)ctx->num_cus * 16;
    uint32_t grid = (uint32_t)(want < cap ? (want ? want : 1) : cap);
    return launch_k(fill_splitmix_kernel, dim3(grid), dim3(256), (hipStream_t)stream, (uint8_t *)d_dst, nbytes, seed,
                    word_offset);
}

int priskv_crc_host_register(void *h_base, uint64_t len)
{
    if (!h_base || !len)
        return -EINVAL;
    return herr(hipHostRegister(h_base, len, hipHostRegisterPortable | hipHostRegisterMapped));
}

int priskv_crc_host_unregister(void *h_base)
{
    if (!h_base)
        return -EINVAL;
    return herr(hipHostUnregister(h_base));
}

namespace {
// Is [h, h + len) one contiguous device-visible mapping (registered or
// pinned)?  Both ends are looked up: a registration that ends inside the
// range would otherwise pass as a mapping of all of it.
// A lookup that fails (an unregistered range) sets the thread's last HIP
// error; it is cleared again only if the caller had no error pending, so a
// server's own earlier error stays visible to its hipGetLastError (HIP has no
// call that restores a specific code: a pending one may read as
// hipErrorInvalidValue afterwards, but it is not lost).
bool host_mapped(const void *h, uint64_t len, void **dptr)
{
    void *d0 = nullptr, *d1 = nullptr;
    const uint8_t *last = (const uint8_t *)h + len - 1;
    const bool pending = hipPeekAtLastError() != hipSuccess;
    const bool ok = hipHostGetDevicePointer(&d0, const_cast<void *>(h), 0) == hipSuccess && d0 &&
                    hipHostGetDevicePointer(&d1, const_cast<uint8_t *>(last), 0) == hipSuccess && d1 &&
                    (uint8_t *)d1 - (uint8_t *)d0 == (ptrdiff_t)(len - 1);
    if (!pending)
        (void)hipGetLastError();
    *dptr = ok ? d0 : nullptr;
    return ok;
}

// Registrations this library makes on the caller's behalf (the zero-copy
// scrub of a region the caller did not register).  One process-wide registry
// of byte ranges: a call whose range lies inside a live temporary
// registration -- several GPUs scrubbing one memfile, the batcher beside a
// scrub, a scrub of a sub-range -- takes a reference on that registration,
// and the last user unregisters it.  A call whose range overlaps a live
// temporary registration without lying inside it waits until that
// registration is gone and then registers its own (pages cannot be
// registered twice).  A caller never waits while it holds a reference, so
// the wait always ends; a new caller whose range overlaps a waiting one
// queues behind it, so a caller that scrubs in a loop cannot keep a waiter
// out.  Check, register and refcount happen under one lock, so no caller can
// see a temporary mapping it reads through disappear.
struct TempReg {
    const uint8_t *base;
    uint64_t len;
    int refs;
};
pthread_mutex_t g_reg_lock = PTHREAD_MUTEX_INITIALIZER;
pthread_cond_t g_reg_gone = PTHREAD_COND_INITIALIZER;
std::vector<TempReg> g_regs;
std::vector<TempReg> g_reg_waiters; // ranges of callers waiting in reg_acquire (refs unused)

bool ranges_overlap(const uint8_t *a, uint64_t alen, const uint8_t *b, uint64_t blen)
{
    return a < b + blen && b < a + alen;
}

// a waiter leaves the queue: new callers it held back may go
void reg_unwait(const uint8_t *b, uint64_t len)
{
    for (size_t i = 0; i < g_reg_waiters.size(); i++)
        if (g_reg_waiters[i].base == b && g_reg_waiters[i].len == len) {
            g_reg_waiters.erase(g_reg_waiters.begin() + (ptrdiff_t)i);
            pthread_cond_broadcast(&g_reg_gone);
            return;
        }
}

// *dptr = device view of [base, base + len); *reg = the temporary
// registration a reference was taken on (release it with reg_release), or
// nullptr when the range is the caller's own registration / pinned memory
int reg_acquire(const void *base, uint64_t len, void **dptr, const void **reg)
{
    *reg = nullptr;
    const uint8_t *b = static_cast<const uint8_t *>(base);
    pthread_mutex_lock(&g_reg_lock);
    bool waiting = false;
    for (;;) {
        const TempReg *cover = nullptr;
        bool blocked = false;
        for (const TempReg &r : g_regs) {
            if (b >= r.base && (uint64_t)(b - r.base) <= r.len && len <= r.len - (uint64_t)(b - r.base))
                cover = &r;
            else if (ranges_overlap(b, len, r.base, r.len))
                blocked = true;
        }
        if (cover) {
            int rc = 0;
            if (host_mapped(base, len, dptr)) {
                const_cast<TempReg *>(cover)->refs++;
                *reg = cover->base;
            } else {
                rc = -EIO;
            }
            if (waiting)
                reg_unwait(b, len);
            pthread_mutex_unlock(&g_reg_lock);
            return rc;
        }
        if (!blocked && !waiting)
            for (const TempReg &w : g_reg_waiters)
                blocked |= ranges_overlap(b, len, w.base, w.len);
        if (!blocked)
            break;
        if (!waiting) {
            try {
                g_reg_waiters.push_back(TempReg{b, len, 0});
            } catch (...) {
                pthread_mutex_unlock(&g_reg_lock);
                return -ENOMEM;
            }
            waiting = true;
        }
        pthread_cond_wait(&g_reg_gone, &g_reg_lock);
    }
    if (waiting)
        reg_unwait(b, len);
    if (host_mapped(base, len, dptr)) { // the caller's own registration / pinned memory
        pthread_mutex_unlock(&g_reg_lock);
        return 0;
    }
    int rc = herr(hipHostRegister(const_cast<void *>(base), len, hipHostRegisterPortable | hipHostRegisterMapped));
    if (!rc && !host_mapped(base, len, dptr)) {
        (void)hipHostUnregister(const_cast<void *>(base));
        rc = -EIO;
    }
    if (!rc) {
        try {
            g_regs.push_back(TempReg{b, len, 1});
            *reg = b;
        } catch (...) {
            (void)hipHostUnregister(const_cast<void *>(base));
            rc = -ENOMEM;
        }
    }
    pthread_mutex_unlock(&g_reg_lock);
    return rc;
}

void reg_release(const void *reg)
{
    if (!reg)
        return;
    pthread_mutex_lock(&g_reg_lock);
    for (size_t i = 0; i < g_regs.size(); i++) {
        if (g_regs[i].base != reg)
            continue;
        if (--g_regs[i].refs == 0) {
            (void)hipHostUnregister(const_cast<uint8_t *>(g_regs[i].base));
            g_regs.erase(g_regs.begin() + (ptrdiff_t)i);
            pthread_cond_broadcast(&g_reg_gone);
        }
        break;
    }
    pthread_mutex_unlock(&g_reg_lock);
}
} // namespace

int priskv_crc32_ranges_host(priskv_crc_ctx *ctx, const void *h_base, uint64_t region_bytes,
                             const uint64_t *h_offsets, const uint32_t *h_lengths, uint64_t n, uint32_t *h_out)
{
    if (!ctx)
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!h_base || !h_offsets || !h_lengths || !h_out || !region_bytes)
        return -EINVAL;
    uint64_t max_len = 1; // known (>= 1): lets launch_extents decide segmentation from the sizes
    for (uint64_t i = 0; i < n; i++) {
        if (h_offsets[i] > region_bytes || h_lengths[i] > region_bytes - h_offsets[i])
            return -EINVAL;
        max_len = h_lengths[i] > max_len ? h_lengths[i] : max_len;
    }
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    // device view of the host mapping (zero-copy): the caller's registration
    // or pinned memory, else a shared temporary registration (reg_acquire)
    void *dptr = nullptr;
    const void *reg = nullptr;
    if (int rc = reg_acquire(h_base, region_bytes, &dptr, &reg))
        return rc;
    pthread_mutex_lock(&ctx->lock);
    int rc = 0;
    const size_t need = (size_t)n * (8 + 4 + 4);
    if (ctx->scrub_cap < need) {
        (void)hipFree(ctx->d_scrub);
        ctx->d_scrub = nullptr;
        ctx->scrub_cap = 0;
        if (!(rc = herr(hipMalloc(&ctx->d_scrub, need))))
            ctx->scrub_cap = need;
    }
    if (!rc) {
        uint64_t *d_off = (uint64_t *)ctx->d_scrub;
        uint32_t *d_len = (uint32_t *)(d_off + n);
        uint32_t *d_crc = d_len + n;
        if (!(rc = herr(hipMemcpyAsync(d_off, h_offsets, n * 8, hipMemcpyHostToDevice, ctx->aux))) &&
            !(rc = herr(hipMemcpyAsync(d_len, h_lengths, n * 4, hipMemcpyHostToDevice, ctx->aux))) &&
            !(rc = ranges_dev(ctx, dptr, d_off, d_len, n, d_crc, ctx->aux, max_len)) &&
            !(rc = herr(hipMemcpyAsync(h_out, d_crc, n * 4, hipMemcpyDeviceToHost, ctx->aux))))
            rc = herr(hipStreamSynchronize(ctx->aux));
        else
            (void)hipStreamSynchronize(ctx->aux);
    }
    pthread_mutex_unlock(&ctx->lock);
    reg_release(reg);
    return rc;
}

// ---- multi-GPU host-resident forms ------------------------------------------
struct MultiJob {
    priskv_crc_ctx *ctx;
    const void *base;
    uint64_t region_bytes;
    const uint64_t *offs;
    const uint32_t *lens;
    uint64_t first, n;
    uint32_t bs;
    uint32_t *out;
    bool ranges;
    int rc;
};

static void *multi_worker(void *arg)
{
    MultiJob *j = (MultiJob *)arg;
    if (!j->n) {
        j->rc = 0;
    } else if (j->ranges) {
        j->rc = priskv_crc32_ranges_host(j->ctx, j->base, j->region_bytes, j->offs + j->first, j->lens + j->first,
                                         j->n, j->out + j->first);
    } else {
        j->rc = priskv_crc32_blocks_host(j->ctx, (const uint8_t *)j->base + j->first * (uint64_t)j->bs, j->n,
                                         j->bs, j->out + j->first);
    }
    return nullptr;
}

static bool valid_ctxs(priskv_crc_ctx *const *ctxs, int nctx)
{
    if (!ctxs || nctx < 1 || nctx > 64)
        return false;
    for (int g = 0; g < nctx; g++) {
        if (!ctxs[g])
            return false;
        for (int h = 0; h < g; h++)
            if (ctxs[g] == ctxs[h])
                return false;
    }
    return true;
}

static int run_multi(priskv_crc_ctx *const *ctxs, int nctx, MultiJob proto, uint64_t n)
{
    if (!valid_ctxs(ctxs, nctx))
        return -EINVAL;
    MultiJob jobs[64];
    pthread_t th[64];
    for (int g = 0; g < nctx; g++) {
        jobs[g] = proto;
        jobs[g].ctx = ctxs[g];
        jobs[g].first = n * (uint64_t)g / (uint64_t)nctx;
        jobs[g].n = n * (uint64_t)(g + 1) / (uint64_t)nctx - jobs[g].first;
        jobs[g].rc = -EIO;
    }
    int started = 1;
    for (int g = 1; g < nctx; g++, started++)
        if (pthread_create(&th[g], nullptr, multi_worker, &jobs[g]))
            break;
    multi_worker(&jobs[0]);
    for (int g = 1; g < started; g++)
        pthread_join(th[g], nullptr);
    for (int g = started; g < nctx; g++) // threads that could not start: run inline
        multi_worker(&jobs[g]);
    for (int g = 0; g < nctx; g++)
        if (jobs[g].rc)
            return jobs[g].rc;
    return 0;
}

int priskv_crc32_blocks_host_multi(priskv_crc_ctx *const *ctxs, int nctx, const void *h_base, uint64_t nblocks,
                                   uint32_t block_size, uint32_t *h_out)
{
    if (block_size == 0 || !valid_ctxs(ctxs, nctx))
        return -EINVAL;
    if (nblocks == 0)
        return 0;
    if (!h_base || !h_out)
        return -EINVAL;
    MultiJob p{};
    p.base = h_base;
    p.bs = block_size;
    p.out = h_out;
    p.ranges = false;
    return run_multi(ctxs, nctx, p, nblocks);
}

int priskv_crc32_ranges_host_multi(priskv_crc_ctx *const *ctxs, int nctx, const void *h_base, uint64_t region_bytes,
                                   const uint64_t *h_offsets, const uint32_t *h_lengths, uint64_t n, uint32_t *h_out)
{
    if (!valid_ctxs(ctxs, nctx))
        return -EINVAL;
    if (n == 0)
        return 0;
    if (!h_base || !h_offsets || !h_lengths || !h_out || !region_bytes)
        return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (h_offsets[i] > region_bytes || h_lengths[i] > region_bytes - h_offsets[i])
            return -EINVAL;
    DevGuard dg(ctxs[0]->device);
    if (!dg.ok)
        return -ENODEV;
    MultiJob p{};
    p.base = h_base;
    p.region_bytes = region_bytes;
    p.offs = h_offsets;
    p.lens = h_lengths;
    p.out = h_out;
    p.ranges = true;
    // one shared registration for all devices (the per-shard calls then find
    // it in the registry instead of each registering the range)
    void *probe = nullptr;
    const void *reg = nullptr;
    if (int rc = reg_acquire(h_base, region_bytes, &probe, &reg))
        return rc;
    const int rc = run_multi(ctxs, nctx, p, n);
    reg_release(reg);
    return rc;
}

// ---- host-streamed path ---------------------------------------------------
// Pageable input is bounced through pinned staging; one core's memcpy caps
// that at ~10-15 GB/s, so the copy is split over PRISKV_CRC_COPY_THREADS
// (default 8) threads.
struct CopyJob {
    void *dst;
    const void *src;
    size_t n;
};

static void *copy_worker(void *arg)
{
    CopyJob *j = (CopyJob *)arg;
    memcpy(j->dst, j->src, j->n);
    return nullptr;
}

static int copy_threads()
{
    static int n = -1;
    if (n < 0) {
        const char *e = getenv("PRISKV_CRC_COPY_THREADS");
        int v = e ? atoi(e) : 8;
        n = v < 1 ? 1 : (v > 32 ? 32 : v);
    }
    return n;
}

static void par_memcpy(void *dst, const void *src, size_t n)
{
    const int T = n >= ((size_t)4 << 20) ? copy_threads() : 1;
    CopyJob jobs[32];
    pthread_t th[32];
    const size_t per = (n / T + 4095) & ~(size_t)4095;
    int started = 0;
    for (int t = 0; t < T; t++) {
        const size_t a = (size_t)t * per;
        jobs[t].dst = (uint8_t *)dst + (a < n ? a : n);
        jobs[t].src = (const uint8_t *)src + (a < n ? a : n);
        jobs[t].n = a < n ? (n - a < per ? n - a : per) : 0;
    }
    for (int t = 1; t < T; t++) {
        if (pthread_create(&th[t], nullptr, copy_worker, &jobs[t]))
            break;
        started = t;
    }
    copy_worker(&jobs[0]);
    for (int t = 1; t <= started; t++)
        pthread_join(th[t], nullptr);
    for (int t = started + 1; t < T; t++)
        copy_worker(&jobs[t]);
}
static int stream_setup(priskv_crc_ctx *c, uint32_t block_size)
{
    size_t want = (size_t)64 << 20; // 64 MiB chunks
    if (want < block_size)
        want = block_size;
    want -= want % block_size;
    if (c->stream_ready && c->chunk_bytes >= want)
        return 0;
    if (c->stream_ready) {
        for (int i = 0; i < NSTREAM; i++) {
            (void)hipStreamSynchronize(c->streams[i]);
            (void)hipStreamDestroy(c->streams[i]);
            (void)hipFree(c->d_stage[i]);
            (void)hipFree(c->d_stage_out[i]);
            (void)hipHostFree(c->h_bounce[i]);
            (void)hipHostFree(c->h_out_stage[i]);
        }
        c->stream_ready = 0;
    }
    memset(c->streams, 0, sizeof(c->streams));
    memset(c->d_stage, 0, sizeof(c->d_stage));
    memset(c->d_stage_out, 0, sizeof(c->d_stage_out));
    memset(c->h_bounce, 0, sizeof(c->h_bounce));
    memset(c->h_out_stage, 0, sizeof(c->h_out_stage));
    const size_t nmax = want / block_size;
    for (int i = 0; i < NSTREAM; i++) {
        int rc;
        if ((rc = herr(hipStreamCreateWithFlags(&c->streams[i], hipStreamNonBlocking))) ||
            (rc = herr(hipMalloc(&c->d_stage[i], want))) ||
            (rc = herr(hipMalloc((void **)&c->d_stage_out[i], nmax * 4))) ||
            (rc = herr(hipHostMalloc(&c->h_bounce[i], want, hipHostMallocDefault))) ||
            (rc = herr(hipHostMalloc((void **)&c->h_out_stage[i], nmax * 4, hipHostMallocDefault))))
            return rc; // partially built state is torn down by ctx_destroy
    }
    c->chunk_bytes = want;
    c->stream_ready = 1;
    return 0;
}

int priskv_crc32_blocks_host(priskv_crc_ctx *ctx, const void *h_base, uint64_t nblocks, uint32_t block_size,
                             uint32_t *h_out)
{
    if (!ctx || block_size == 0)
        return -EINVAL;
    if (nblocks == 0)
        return 0;
    if (!h_base || !h_out)
        return -EINVAL;
    DevGuard g(ctx->device);
    if (!g.ok)
        return -ENODEV;
    pthread_mutex_lock(&ctx->lock);
    int rc = stream_setup(ctx, block_size);
    if (rc) {
        pthread_mutex_unlock(&ctx->lock);
        return rc;
    }
    // pinned / registered input is DMA'd directly; pageable input bounces
    // (the whole batch, both ends: a registration that stops short of the
    // last block would have the DMA read unpinned pages)
    void *dview = nullptr;
    const bool pinned = host_mapped(h_base, nblocks * (uint64_t)block_size, &dview);
    const uint64_t per = ctx->chunk_bytes / block_size;
    const uint64_t nchunks = (nblocks + per - 1) / per;
    uint64_t pending_first[NSTREAM], pending_n[NSTREAM];
    for (int i = 0; i < NSTREAM; i++)
        pending_n[i] = 0;
    for (uint64_t ci = 0; ci < nchunks && !rc; ci++) {
        const int sl = (int)(ci % NSTREAM);
        hipStream_t s = ctx->streams[sl];
        if (pending_n[sl]) { // recycle the slot: drain it and hand its results out
            if ((rc = herr(hipStreamSynchronize(s))))
                break;
            memcpy(h_out + pending_first[sl], ctx->h_out_stage[sl], pending_n[sl] * 4);
            pending_n[sl] = 0;
        }
        const uint64_t first = ci * per;
        const uint64_t nb = (nblocks - first < per) ? nblocks - first : per;
        const uint8_t *src = (const uint8_t *)h_base + first * block_size;
        const size_t bytes = (size_t)(nb * block_size);
        if (!pinned) {
            par_memcpy(ctx->h_bounce[sl], src, bytes);
            src = (const uint8_t *)ctx->h_bounce[sl];
        }
        if ((rc = herr(hipMemcpyAsync(ctx->d_stage[sl], src, bytes, hipMemcpyHostToDevice, s))))
            break;
        if ((rc = launch_blocks(ctx, (const uint8_t *)ctx->d_stage[sl], nb, block_size, ctx->d_stage_out[sl], s)))
            break;
        if ((rc = herr(hipMemcpyAsync(ctx->h_out_stage[sl], ctx->d_stage_out[sl], nb * 4, hipMemcpyDeviceToHost, s))))
            break;
        pending_first[sl] = first;
        pending_n[sl] = nb;
    }
    for (int sl = 0; sl < NSTREAM; sl++) {
        int r2 = herr(hipStreamSynchronize(ctx->streams[sl]));
        if (!rc && r2)
            rc = r2;
        if (!rc && pending_n[sl])
            memcpy(h_out + pending_first[sl], ctx->h_out_stage[sl], pending_n[sl] * 4);
    }
    pthread_mutex_unlock(&ctx->lock);
    return rc;
}

} // extern "C"
