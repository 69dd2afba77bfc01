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

#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/priskv_crc_gpu.h"
#include "crc_internal.h"

#define PRV_VERSION "priskv-crc-mi355x 0.1 (gfx950)"

namespace {

constexpr int kWaves = 8;                 // waves per workgroup
constexpr int kThreads = kWaves * 64;     // 512
constexpr int kLdsWords = PRV_LDS_WORDS;  // 16384 words = 64 KiB
constexpr int kSetB = 128;                // byte offset of set B inside an LDS row
constexpr int kFoldSets = 7;              // G = 1,2,4,...,64

__shared__ uint32_t s_tab[kLdsWords];

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
struct LaneConst {
    uint32_t c;                  // byte i = 16k + 4t_i  (LDS column of instruction i)
    uint32_t s0, s1, s2, s3;     // v_perm selectors of instruction i
};

__device__ __forceinline__ LaneConst lane_const(int lane)
{
    LaneConst L;
    const uint32_t k = (lane >> 2) & 7;
    uint32_t c = 0, s[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t t = (i + lane) & 3;
        c |= (16u * k + 4u * t) << (8 * i);
        // result byte0 <- c byte i (S1 bytes 0-3), byte1 <- x byte t (S0 bytes
        // 4-7), bytes 2,3 <- 0x00 (selector 0x0c)
        s[i] = 0x0c0c0000u | ((4u + t) << 8) | (uint32_t)i;
    }
    L.c = c;
    L.s0 = s[0];
    L.s1 = s[1];
    L.s2 = s[2];
    L.s3 = s[3];
    return L;
}

template <int SETOFF>
__device__ __forceinline__ uint32_t zstep(uint32_t x, const LaneConst &L)
{
    const uint32_t a0 = __builtin_amdgcn_perm(x, L.c, L.s0);
    const uint32_t a1 = __builtin_amdgcn_perm(x, L.c, L.s1);
    const uint32_t a2 = __builtin_amdgcn_perm(x, L.c, L.s2);
    const uint32_t a3 = __builtin_amdgcn_perm(x, L.c, L.s3);
    const char *t = reinterpret_cast<const char *>(s_tab) + SETOFF;
    const uint32_t r0 = *reinterpret_cast<const uint32_t *>(t + a0);
    const uint32_t r1 = *reinterpret_cast<const uint32_t *>(t + a1);
    const uint32_t r2 = *reinterpret_cast<const uint32_t *>(t + a2);
    const uint32_t r3 = *reinterpret_cast<const uint32_t *>(t + a3);
    return r0 ^ r1 ^ r2 ^ r3;
}

// one 16-byte piece; LAST = this piece ends the lane's part of the block
template <bool LAST>
__device__ __forceinline__ uint32_t piece(uint32_t u, const v4u &d, const LaneConst &L)
{
    u = zstep<0>(u ^ d.x, L);
    u = zstep<0>(u ^ d.y, L);
    u = zstep<0>(u ^ d.z, L);
    return LAST ? zstep<0>(u ^ d.w, L) : zstep<kSetB>(u ^ d.w, L);
}

// v -> sum_i bit_i(v) * col[i]   (per-lane GF(2) matrix-vector)
__device__ __forceinline__ uint32_t bitmat(uint32_t v, const uint32_t (&col)[32])
{
    uint32_t f = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const uint32_t m = (uint32_t)(((int32_t)(v << (31 - i))) >> 31);
        f ^= m & col[i];
    }
    return f;
}

__device__ __forceinline__ uint32_t dpp_xor(uint32_t v, int ctrl_sel)
{
    // ctrl is a compile-time constant at every call site
    switch (ctrl_sel) {
    case 0: return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
    case 1: return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
    case 2: return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    default: return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false); // row_ror:8
    }
}

// XOR over all 64 lanes; result is wave-uniform
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
    v = dpp_xor(v, 0);
    v = dpp_xor(v, 1);
    v = dpp_xor(v, 2);
    v = dpp_xor(v, 3);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// XOR within aligned groups of G lanes (G power of two <= 64); every lane of
// a group ends with the group total
template <int G>
__device__ __forceinline__ uint32_t group_xor(uint32_t v)
{
#pragma unroll
    for (int m = 1; m < G; m <<= 1)
        v ^= (uint32_t)__shfl_xor((int)v, m, 64);
    return v;
}

__device__ __forceinline__ void load_lds_image(const uint32_t *__restrict__ img)
{
    const uint4 *src = reinterpret_cast<const uint4 *>(img);
    uint4 *dst = reinterpret_cast<uint4 *>(s_tab);
    for (int i = threadIdx.x; i < kLdsWords / 4; i += blockDim.x)
        dst[i] = src[i];
}

// Buffer loads through a wave-uniform descriptor: the chunk base lives in
// SGPRs (rebuilt per chunk with scalar ops), the lane offset is the voffset
// VGPR and the row offset the 12-bit immediate -- no 64-bit VALU address
// math in the loop (T8/T20 of the CDNA HIP guide).  aux 2 = nt (streamed once).
template <int CH>
__device__ __forceinline__ void load_chunk(v4u (&X)[CH], const uint8_t *wp, uint32_t loff)
{
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(wp), 0, CH * PRV_ROW_BYTES, 0x00020000);
#pragma unroll
    for (int k = 0; k < CH; k++)
        X[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(loff + k * PRV_ROW_BYTES), 0, 2));
}

// ---------------------------------------------------------------------------
// hot kernel: block_size = R KiB (R % CH == 0), base 16-byte aligned.
// Waves own contiguous block ranges; chunks of CH rows are double-buffered in
// registers so the next chunk's loads are in flight while this one is hashed.
// ---------------------------------------------------------------------------
template <int CH>
__device__ __forceinline__ uint32_t hash_chunk(uint32_t u, const v4u (&X)[CH], bool seg_end,
                                               const LaneConst &L, const uint32_t (&col)[32],
                                               uint32_t &res, uint32_t &nres, uint64_t &res_base,
                                               uint32_t *__restrict__ out, int lane)
{
#pragma unroll
    for (int k = 0; k < CH - 1; k++)
        u = piece<false>(u, X[k], L);
    if (!seg_end)
        return piece<false>(u, X[CH - 1], L);
    u = piece<true>(u, X[CH - 1], L);
    const uint32_t crc = wave_xor(bitmat(u, col));
    res = (lane == (int)nres) ? crc : res;
    if (++nres == 64) {
        out[res_base + lane] = res;
        res_base += 64;
        nres = 0;
    }
    return 0;
}

template <int CH>
__global__ __launch_bounds__(kThreads, 4) void crc_rows_kernel(
    const uint8_t *__restrict__ base, uint64_t nblocks, uint32_t rows_per_block,
    const uint32_t *__restrict__ lds_image, const uint32_t *__restrict__ fold64,
    uint32_t *__restrict__ out)
{
    load_lds_image(lds_image);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneConst L = lane_const(lane);
    uint32_t col[32];
#pragma unroll
    for (int i = 0; i < 32; i++)
        col[i] = fold64[i * 64 + lane];
    __syncthreads();

    const uint64_t W = (uint64_t)gridDim.x * kWaves;
    const uint64_t wid = (uint64_t)blockIdx.x * kWaves + wave;
    const uint64_t b0 = nblocks * wid / W;
    const uint64_t b1 = nblocks * (wid + 1) / W;
    if (b0 >= b1)
        return;
    const uint32_t cps = rows_per_block / CH;            // chunks per block
    const uint32_t nq = (uint32_t)(b1 - b0) * cps;       // chunks of this wave (< 2^32: host-checked)
    const uint64_t chunk_bytes = (uint64_t)CH * PRV_ROW_BYTES;
    const uint8_t *wp = base + b0 * (uint64_t)rows_per_block * PRV_ROW_BYTES; // wave-uniform
    const uint32_t loff = (uint32_t)lane * 16;

    // software pipeline: chunk q+1's loads are issued (and pinned there by a
    // scheduling barrier) before chunk q is hashed
    v4u A[CH], B[CH];
    load_chunk<CH>(A, wp, loff);
    uint32_t u = 0, cq = 0, res = 0, nres = 0;
    uint64_t res_base = b0;
    for (uint32_t q = 0;;) {
        // always issue (clamped to the last chunk) so the waitcnt before the
        // hash below counts only the older chunk's loads on every path
        load_chunk<CH>(B, wp + (uint64_t)(q + 1 < nq ? q + 1 : q) * chunk_bytes, loff);
        __builtin_amdgcn_sched_barrier(0);
        u = hash_chunk<CH>(u, A, cq + 1 == cps, L, col, res, nres, res_base, out, lane);
        cq = (cq + 1 == cps) ? 0 : cq + 1;
        if (++q >= nq)
            break;
        load_chunk<CH>(A, wp + (uint64_t)(q + 1 < nq ? q + 1 : q) * chunk_bytes, loff);
        __builtin_amdgcn_sched_barrier(0);
        u = hash_chunk<CH>(u, B, cq + 1 == cps, L, col, res, nres, res_base, out, lane);
        cq = (cq + 1 == cps) ? 0 : cq + 1;
        if (++q >= nq)
            break;
    }
    if (nres && lane < (int)nres)
        out[res_base + lane] = res;
}

// ---------------------------------------------------------------------------
// sub-KiB power-of-two blocks (16..512 B): G = block/16 lanes per block, one
// 1 KiB row holds 64/G blocks; no row gap, per-lane fold over Z_(16(G-1-l%G)).
// ---------------------------------------------------------------------------
template <int G>
__global__ __launch_bounds__(kThreads, 4) void crc_small_kernel(
    const uint8_t *__restrict__ base, uint64_t nblocks, const uint32_t *__restrict__ lds_image,
    const uint32_t *__restrict__ foldG, uint32_t *__restrict__ out)
{
    load_lds_image(lds_image);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneConst L = lane_const(lane);
    uint32_t col[32];
#pragma unroll
    for (int i = 0; i < 32; i++)
        col[i] = foldG[i * 64 + lane];
    __syncthreads();

    constexpr uint32_t kBlock = 16u * G;
    constexpr uint32_t kPerRow = 64 / G;
    const uint64_t nrows = (nblocks + kPerRow - 1) / kPerRow;
    const uint64_t W = (uint64_t)gridDim.x * kWaves;
    const uint64_t wid = (uint64_t)blockIdx.x * kWaves + wave;
    const uint64_t r0 = nrows * wid / W, r1 = nrows * (wid + 1) / W;
    for (uint64_t r = r0; r < r1; r += 4) {
        v4u X[4];
        bool ok[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t blk = (r + k) * kPerRow + lane / G;
            ok[k] = (r + k < r1) && (blk < nblocks);
            X[k] = ok[k] ? *reinterpret_cast<const v4u *>(base + blk * kBlock + (lane % G) * 16)
                         : v4u{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (r + k >= r1)
                break;
            const uint32_t crc = group_xor<G>(bitmat(piece<true>(0u, X[k], L), col));
            const uint64_t blk = (r + k) * kPerRow + lane / G;
            if (ok[k] && (lane % G) == 0)
                out[blk] = crc;
        }
    }
}

// ---------------------------------------------------------------------------
// generic path: any size / alignment.  One thread per item, byte-serial
// Sarwate steps (server/crc.c:70-73) against a single LDS table.  Used for
// odd block sizes and for per-value (offset, length) extents.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void crc_generic_kernel(
    const uint8_t *__restrict__ base, uint64_t n, uint64_t stride, uint32_t len_const,
    const uint64_t *__restrict__ offsets, const uint32_t *__restrict__ lengths,
    const uint32_t *__restrict__ sarwate, uint32_t *__restrict__ out)
{
    __shared__ uint32_t t[256];
    t[threadIdx.x] = sarwate[threadIdx.x];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *p = base + (offsets ? offsets[i] : i * stride);
        uint32_t len = lengths ? lengths[i] : len_const;
        uint32_t crc = 0;
        // align to 4 bytes, then consume words (still one table step per byte)
        while (len && ((uintptr_t)p & 3)) {
            crc = t[(crc ^ *p++) & 0xff] ^ (crc >> 8);
            len--;
        }
        while (len >= 4) {
            uint32_t w = *reinterpret_cast<const uint32_t *>(p);
            crc ^= w;
            crc = t[crc & 0xff] ^ (crc >> 8);
            crc = t[crc & 0xff] ^ (crc >> 8);
            crc = t[crc & 0xff] ^ (crc >> 8);
            crc = t[crc & 0xff] ^ (crc >> 8);
            p += 4;
            len -= 4;
        }
        while (len--)
            crc = t[(crc ^ *p++) & 0xff] ^ (crc >> 8);
        out[i] = crc;
    }
}

// ---------------------------------------------------------------------------
// test-pattern fill: 64-bit word i = splitmix64(seed + (off + i + 1) * phi)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t *__restrict__ dst, uint64_t nbytes,
                                                            uint64_t seed, uint64_t word_offset)
{
    const uint64_t nw2 = nbytes / 16; // pairs of words
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw2;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = word_offset + 2 * i;
        const uint64_t a = mix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
        const uint64_t b = mix64(seed + (w + 2) * 0x9E3779B97F4A7C15ull);
        v4u v = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
        __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(dst + 16 * i));
    }
    if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) {
        const uint64_t pos = (nbytes & ~(uint64_t)15) + threadIdx.x;
        const uint64_t w = word_offset + pos / 8;
        const uint64_t v = mix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
        dst[pos] = (uint8_t)(v >> (8 * (pos & 7)));
    }
}

} // namespace

// ===========================================================================
// host shim
// ===========================================================================
#define NSTREAM 3

struct priskv_crc_ctx {
    int device;
    int num_cus;
    int max_wgs;               // resident workgroups of the rows kernel (2 per CU)
    uint32_t *d_lds_image;     // 64 KiB
    uint32_t *d_fold;          // kFoldSets x 2048 words, set j for G = 1 << j
    uint32_t *d_sarwate;       // 256 words
    // host-streamed path (guarded by lock)
    pthread_mutex_t lock;
    int stream_ready;
    size_t chunk_bytes;
    hipStream_t streams[NSTREAM];
    void *d_stage[NSTREAM];
    uint32_t *d_stage_out[NSTREAM];
    void *h_bounce[NSTREAM];
    uint32_t *h_out_stage[NSTREAM];
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

inline int herr(hipError_t e)
{
    if (e == hipSuccess)
        return 0;
    if (e == hipErrorOutOfMemory)
        return -ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice)
        return -ENODEV;
    return -EIO;
}

inline bool is_pow2(uint64_t v) { return v && !(v & (v - 1)); }

enum Path { PATH_ROWS = 1, PATH_ROWS_COOP = 2, PATH_SMALL = 3, PATH_GENERIC = 4 };

int choose_path(const void *d_base, uint32_t block_size)
{
    const bool aligned = ((uintptr_t)d_base & 15) == 0;
    if (aligned && block_size % PRV_ROW_BYTES == 0)
        return PATH_ROWS;
    if (aligned && is_pow2(block_size) && block_size >= 16 && block_size <= 512)
        return PATH_SMALL;
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
    hipLaunchKernelGGL(crc_generic_kernel, dim3(grid), dim3(256), 0, s, base, n, stride, len_const, offs,
                       lens, ctx->d_sarwate, out);
    return herr(hipGetLastError());
}

int launch_blocks(const priskv_crc_ctx *ctx, const uint8_t *base, uint64_t nblocks, uint32_t bs,
                  uint32_t *out, hipStream_t s)
{
    const int path = choose_path(base, bs);
    if (path == PATH_ROWS) {
        const uint32_t R = bs / PRV_ROW_BYTES;
        const int ch = (R % 4 == 0) ? 4 : (R % 2 == 0 ? 2 : 1);
        const uint64_t cps = R / ch;
        // the kernel counts a wave's chunks in 32 bits: cap blocks per launch
        const uint64_t waves = (uint64_t)ctx->max_wgs * kWaves;
        const uint64_t cap = waves * ((1ull << 31) / cps - 1);
        for (uint64_t done = 0; done < nblocks;) {
            const uint64_t n = (nblocks - done < cap) ? nblocks - done : cap;
            const uint64_t want = (n + kWaves - 1) / kWaves;
            const uint32_t grid = (uint32_t)(want < (uint64_t)ctx->max_wgs ? want : (uint64_t)ctx->max_wgs);
            const uint8_t *b = base + done * bs;
            uint32_t *o = out + done;
            if (ch == 4)
                hipLaunchKernelGGL(crc_rows_kernel<4>, dim3(grid), dim3(kThreads), 0, s, b, n, R,
                                   ctx->d_lds_image, ctx->d_fold + 6 * 2048, o);
            else if (ch == 2)
                hipLaunchKernelGGL(crc_rows_kernel<2>, dim3(grid), dim3(kThreads), 0, s, b, n, R,
                                   ctx->d_lds_image, ctx->d_fold + 6 * 2048, o);
            else
                hipLaunchKernelGGL(crc_rows_kernel<1>, dim3(grid), dim3(kThreads), 0, s, b, n, R,
                                   ctx->d_lds_image, ctx->d_fold + 6 * 2048, o);
            if (int rc = herr(hipGetLastError()))
                return rc;
            done += n;
        }
        return 0;
    }
    if (path == PATH_SMALL) {
        const int g = log2u(bs / 16); // G = 1 << g
        const uint64_t rows = (nblocks * bs + PRV_ROW_BYTES - 1) / PRV_ROW_BYTES;
        uint64_t want = (rows + 4 * kWaves - 1) / (4 * kWaves);
        uint32_t grid = (uint32_t)(want < (uint64_t)ctx->max_wgs ? want : (uint64_t)ctx->max_wgs);
        if (grid == 0)
            grid = 1;
        const uint32_t *fold = ctx->d_fold + g * 2048;
        switch (g) {
        case 0: hipLaunchKernelGGL(crc_small_kernel<1>, dim3(grid), dim3(kThreads), 0, s, base, nblocks, ctx->d_lds_image, fold, out); break;
        case 1: hipLaunchKernelGGL(crc_small_kernel<2>, dim3(grid), dim3(kThreads), 0, s, base, nblocks, ctx->d_lds_image, fold, out); break;
        case 2: hipLaunchKernelGGL(crc_small_kernel<4>, dim3(grid), dim3(kThreads), 0, s, base, nblocks, ctx->d_lds_image, fold, out); break;
        case 3: hipLaunchKernelGGL(crc_small_kernel<8>, dim3(grid), dim3(kThreads), 0, s, base, nblocks, ctx->d_lds_image, fold, out); break;
        case 4: hipLaunchKernelGGL(crc_small_kernel<16>, dim3(grid), dim3(kThreads), 0, s, base, nblocks, ctx->d_lds_image, fold, out); break;
        default: hipLaunchKernelGGL(crc_small_kernel<32>, dim3(grid), dim3(kThreads), 0, s, base, nblocks, ctx->d_lds_image, fold, out); break;
        }
        return herr(hipGetLastError());
    }
    return launch_generic(ctx, base, nblocks, bs, bs, nullptr, nullptr, out, s);
}

} // namespace

extern "C" {

const char *priskv_crc_version(void) { return PRV_VERSION; }

int priskv_crc32_blocks_path(const void *d_base, uint64_t nblocks, uint32_t block_size)
{
    if (block_size == 0 || (nblocks && !d_base))
        return -EINVAL;
    return choose_path(d_base, block_size);
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
    int rc = 0;
    uint32_t *h_img = (uint32_t *)malloc(sizeof(uint32_t) * PRV_LDS_WORDS);
    uint32_t *h_fold = (uint32_t *)malloc(sizeof(uint32_t) * 2048 * kFoldSets);
    uint32_t h_sar[256];
    if (!h_img || !h_fold) {
        rc = -ENOMEM;
        goto fail;
    }
    if ((rc = herr(hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, device))))
        goto fail;
    c->max_wgs = 2 * c->num_cus;
    prv_lds_image(h_img, PRV_ROW_GAP);
    for (int j = 0; j < kFoldSets; j++)
        prv_fold_columns(h_fold + j * 2048, 1u << j);
    prv_sarwate_table(h_sar);
    if ((rc = herr(hipMalloc((void **)&c->d_lds_image, sizeof(uint32_t) * PRV_LDS_WORDS))) ||
        (rc = herr(hipMalloc((void **)&c->d_fold, sizeof(uint32_t) * 2048 * kFoldSets))) ||
        (rc = herr(hipMalloc((void **)&c->d_sarwate, sizeof(h_sar)))))
        goto fail;
    if ((rc = herr(hipMemcpy(c->d_lds_image, h_img, sizeof(uint32_t) * PRV_LDS_WORDS, hipMemcpyHostToDevice))) ||
        (rc = herr(hipMemcpy(c->d_fold, h_fold, sizeof(uint32_t) * 2048 * kFoldSets, hipMemcpyHostToDevice))) ||
        (rc = herr(hipMemcpy(c->d_sarwate, h_sar, sizeof(h_sar), hipMemcpyHostToDevice))))
        goto fail;
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
    (void)hipFree(c->d_lds_image);
    (void)hipFree(c->d_fold);
    (void)hipFree(c->d_sarwate);
    pthread_mutex_destroy(&c->lock);
    free(c);
}

int priskv_crc_ctx_device(const priskv_crc_ctx *ctx) { return ctx ? ctx->device : -EINVAL; }

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

int priskv_crc32_ranges_dev(const priskv_crc_ctx *ctx, const void *d_base, const uint64_t *d_offsets,
                            const uint32_t *d_lengths, uint64_t n, uint32_t *d_out, void *stream)
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
    return launch_generic(ctx, (const uint8_t *)d_base, n, 0, 0, d_offsets, d_lengths, d_out,
                          (hipStream_t)stream);
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
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint8_t *)d_dst,
                       nbytes, seed, word_offset);
    return herr(hipGetLastError());
}

int priskv_crc_host_register(void *h_base, uint64_t len)
{
    if (!h_base || !len)
        return -EINVAL;
    return herr(hipHostRegister(h_base, len, hipHostRegisterDefault));
}

int priskv_crc_host_unregister(void *h_base)
{
    if (!h_base)
        return -EINVAL;
    return herr(hipHostUnregister(h_base));
}

// ---- host-streamed path ---------------------------------------------------
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
    bool pinned = false;
    {
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, h_base) == hipSuccess && attr.type == hipMemoryTypeHost)
            pinned = true;
        (void)hipGetLastError();
    }
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
            memcpy(ctx->h_bounce[sl], src, bytes);
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
