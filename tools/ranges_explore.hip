// ranges_explore.hip -- design-space explorer for the extents kernel (not product).
//
// Times crc_ranges_kernel<CH, NBUF, AUX> variants and workgroups per CU,
// interleaved round-robin in one process, on four extent sets:
//   priskv  values as PrisKV places them (random 4 KiB block, 1/2/4 blocks,
//           ragged last block: server/buddy.c:134-140), in request order;
//   sorted  the same extents sorted by offset (scrub order);
//   s4100   fixed 4100-B extents back to back (unaligned block batches);
//   s4096   fixed 4096-B aligned extents (compare: rows kernel on 4 KiB);
//   s65600, s1Mp100  large fixed-length extents, unaligned;
// checking every variant bit-exactly against the first.
// Usage: ranges_explore [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <random>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../priskv_amd/csrc/crc_internal.h"

namespace {
#include "../priskv_amd/csrc/crc_device.inc"
} // namespace

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

typedef void (*LaunchFn)(dim3, const uint8_t *, uint64_t, const uint64_t *, const uint32_t *, uint64_t, uint32_t,
                         const uint32_t *, const uint32_t *, const uint32_t *, uint32_t *);

struct Variant {
    const char *name;
    int wg_per_cu;
    LaunchFn launch;
    bool g32; // two-stream kernel: G = 32 tables and fold columns
};

#define RV(CH, NB, AUX, WG)                                                                                    \
    Variant{"ext CH" #CH " NBUF" #NB " AUX" #AUX " wg/cu" #WG, WG,                                             \
            [](dim3 g, const uint8_t *b, uint64_t n, const uint64_t *o, const uint32_t *l, uint64_t stride,       \
               uint32_t lc, const uint32_t *img, const uint32_t *fold, const uint32_t *un, uint32_t *out) {       \
                hipLaunchKernelGGL((crc_ranges_kernel<CH, NB, AUX>), g, dim3(kThreads), 0, 0, b, n, o, l, 0ull,   \
                                   stride, lc, img, fold, un, out, nullptr, nullptr, nullptr, nullptr);                              \
            }, false}

// OPT bit 0 (nibble fold) takes its two images from these globals
static uint32_t *g_nib16 = nullptr, *g_rowshift = nullptr;
#define RVO(CH, NB, AUX, WG, OPT)                                                                              \
    Variant{"ext CH" #CH " NBUF" #NB " AUX" #AUX " wg/cu" #WG " opt" #OPT, WG,                                 \
            [](dim3 g, const uint8_t *b, uint64_t n, const uint64_t *o, const uint32_t *l, uint64_t stride,       \
               uint32_t lc, const uint32_t *img, const uint32_t *fold, const uint32_t *un, uint32_t *out) {       \
                hipLaunchKernelGGL((crc_ranges_kernel<CH, NB, AUX, OPT>), g, dim3(kThreads), 0, 0, b, n, o, l,     \
                                   0ull, stride, lc, img, ((OPT) & 1) ? g_nib16 : fold,                           \
                                   ((OPT) & 1) ? g_rowshift : un, out, nullptr, nullptr, nullptr, nullptr);                         \
            }, false}

// one 16-wave workgroup per CU (OPT bit 10)
#define RVO16(CH, NB, AUX, OPT)                                                                                \
    Variant{"ext CH" #CH " NBUF" #NB " AUX" #AUX " 16 waves opt" #OPT, 1,                                       \
            [](dim3 g, const uint8_t *b, uint64_t n, const uint64_t *o, const uint32_t *l, uint64_t stride,       \
               uint32_t lc, const uint32_t *img, const uint32_t *fold, const uint32_t *un, uint32_t *out) {       \
                hipLaunchKernelGGL((crc_ranges_kernel<CH, NB, AUX, (OPT) | 1024>), g, dim3(1024), 0, 0, b, n, o, l, \
                                   0ull, stride, lc, img, ((OPT) & 1) ? g_nib16 : fold,                           \
                                   ((OPT) & 1) ? g_rowshift : un, out, nullptr, nullptr, nullptr, nullptr);       \
            }, false}

// 16-wave workgroups, WG of them per CU (OPT without progress priority fits
// two 80 KiB workgroups in the CU's 160 KiB of LDS)
#define RVO16W(CH, NB, AUX, OPT, WG)                                                                          \
    Variant{"ext CH" #CH " NBUF" #NB " AUX" #AUX " 16 waves x" #WG " opt" #OPT, WG,                             \
            [](dim3 g, const uint8_t *b, uint64_t n, const uint64_t *o, const uint32_t *l, uint64_t stride,       \
               uint32_t lc, const uint32_t *img, const uint32_t *fold, const uint32_t *un, uint32_t *out) {       \
                hipLaunchKernelGGL((crc_ranges_kernel<CH, NB, AUX, (OPT) | 1024>), g, dim3(1024), 0, 0, b, n, o, l, \
                                   0ull, stride, lc, img, g_nib16, g_rowshift, out, nullptr, nullptr, nullptr,     \
                                   nullptr);                                                                      \
            }, false}

struct Set {
    const char *name;
    uint64_t n, stride;
    uint32_t len_const;
    uint64_t *d_off = nullptr;
    uint32_t *d_len = nullptr;
    double bytes = 0;
};

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t region = 4ull << 30;
    uint8_t *d;
    CK(hipMalloc(&d, region + 4096));
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(ncu * 16), dim3(256), 0, 0, d, region + 4096, 0x5EED5EEDull, 0ull);

    std::vector<uint32_t> img(PRV_LDS_WORDS), fold(2048), un(16 * 32);
    prv_lds_image(img.data(), 1008);
    prv_fold_columns(fold.data(), 64);
    prv_unshift_columns(un.data());
    std::vector<uint32_t> img32(PRV_LDS_WORDS), fold32(2048);
    prv_lds_image(img32.data(), 496);
    prv_fold_columns(fold32.data(), 32);
    uint32_t *d_img32, *d_fold32;
    CK(hipMalloc(&d_img32, img32.size() * 4));
    CK(hipMalloc(&d_fold32, fold32.size() * 4));
    CK(hipMemcpy(d_img32, img32.data(), img32.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_fold32, fold32.data(), fold32.size() * 4, hipMemcpyHostToDevice));
    uint32_t *d_img, *d_fold, *d_un;
    CK(hipMalloc(&d_img, img.size() * 4));
    CK(hipMalloc(&d_fold, fold.size() * 4));
    CK(hipMalloc(&d_un, un.size() * 4));
    CK(hipMemcpy(d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_fold, fold.data(), fold.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_un, un.data(), un.size() * 4, hipMemcpyHostToDevice));
    {
        std::vector<uint32_t> nib(8 * 16 * 16), rs(16 * 4 * 32);
        prv_fold_nibbles(nib.data(), 16, 16);
        prv_rowshift_columns(rs.data());
        CK(hipMalloc(&g_nib16, nib.size() * 4));
        CK(hipMalloc(&g_rowshift, rs.size() * 4));
        CK(hipMemcpy(g_nib16, nib.data(), nib.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(g_rowshift, rs.data(), rs.size() * 4, hipMemcpyHostToDevice));
    }

    // PrisKV-shaped extents (as tools/bench_paths.py extents())
    const uint64_t n = 1 << 19, bs = 4096;
    std::mt19937_64 rng(1);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t span = (1ull << (rng() % 3)) * bs;
        const uint64_t blk = rng() % (region / bs - 4);
        off[i] = blk * bs;
        len[i] = (uint32_t)std::min<uint64_t>(span - rng() % bs, region - off[i]);
    }
    std::vector<Set> sets;
    auto add = [&](const char *name, const std::vector<uint64_t> &o, const std::vector<uint32_t> &l) {
        Set s{name, o.size(), 0, 0};
        CK(hipMalloc(&s.d_off, o.size() * 8));
        CK(hipMalloc(&s.d_len, l.size() * 4));
        CK(hipMemcpy(s.d_off, o.data(), o.size() * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(s.d_len, l.data(), l.size() * 4, hipMemcpyHostToDevice));
        for (auto v : l)
            s.bytes += v;
        sets.push_back(s);
    };
    add("priskv", off, len);
    if (getenv("RANGES_PK64K")) { // PrisKV-shaped values on 64 KiB blocks (few per wave)
        const uint64_t n64 = 1 << 15, bs64 = 65536;
        std::vector<uint64_t> o1(n64);
        std::vector<uint32_t> l1(n64);
        for (uint64_t i = 0; i < n64; i++) {
            const uint64_t span = (1ull << (rng() % 3)) * bs64;
            const uint64_t blk = rng() % (region / bs64 - 4);
            o1[i] = blk * bs64;
            l1[i] = (uint32_t)std::min<uint64_t>(span - rng() % bs64, region - o1[i]);
        }
        add("pk64k", o1, l1);
    }
    if (getenv("RANGES_SPANS")) { // PrisKV-shaped values of one span each: 1, 2, 4 blocks
        for (int sp = 0; sp < 3; sp++) {
            std::vector<uint64_t> o1(n);
            std::vector<uint32_t> l1(n);
            for (uint64_t i = 0; i < n; i++) {
                const uint64_t span = (1ull << sp) * bs;
                const uint64_t blk = rng() % (region / bs - 4);
                o1[i] = blk * bs;
                l1[i] = (uint32_t)std::min<uint64_t>(span - rng() % bs, region - o1[i]);
            }
            static const char *nm[3] = {"span1", "span2", "span4"};
            add(nm[sp], o1, l1);
        }
    }
    {
        std::vector<uint64_t> idx(n);
        std::iota(idx.begin(), idx.end(), 0);
        std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return off[a] < off[b]; });
        std::vector<uint64_t> o2(n);
        std::vector<uint32_t> l2(n);
        for (uint64_t i = 0; i < n; i++) {
            o2[i] = off[idx[i]];
            l2[i] = len[idx[i]];
        }
        add("sorted", o2, l2);
    }
    {
        Set s{"s4100", region / 4100, 4100, 4100};
        s.bytes = (double)s.n * 4100;
        sets.push_back(s);
        Set t{"s4096", region / 4096, 4096, 4096};
        t.bytes = (double)t.n * 4096;
        sets.push_back(t);
        Set u{"s65600", region / 65600, 65600, 65600};
        u.bytes = (double)u.n * 65600;
        sets.push_back(u);
        Set w{"s1Mp100", region / ((1 << 20) + 100), (1 << 20) + 100, (1 << 20) + 100};
        w.bytes = (double)w.n * ((1 << 20) + 100);
        sets.push_back(w);
    }

    std::vector<Variant> V = {RVO(2, 2, 2, 2, 3),         RVO16(2, 2, 2, 3),       RVO16(2, 2, 2, 3 | 256),
                              RVO16(2, 2, 2, 3 | 512),    RVO16(2, 2, 2, 3 | 768)};
    if (getenv("RANGES_R3")) // round 3: product, skipped virtual rows (8192), read roof (4096), shapes
        V = {RVO16(2, 2, 2, 3 | 768),        RVO16(2, 2, 2, 3 | 768 | 8192), RVO16(2, 2, 2, 3 | 768 | 4096),
             RVO16(2, 3, 2, 3 | 768 | 8192), RVO16(4, 2, 2, 3 | 768 | 8192), RVO16(1, 4, 2, 3 | 768 | 8192),
             RVO16(2, 3, 2, 3 | 768 | 4096), RVO16(4, 2, 2, 3 | 768 | 4096), RVO16W(2, 2, 2, 3 | 8192, 2),
             RVO16W(2, 3, 2, 3 | 8192, 2), RVO16W(2, 2, 2, 3 | 4096, 2)};
    if (getenv("RANGES_R3B")) // round 3: chunk shapes of the many-extents launch shape
        V = {RVO16(2, 2, 2, 3 | 768),        RVO16(4, 2, 2, 3 | 768),        RVO16(4, 3, 2, 3 | 768),
             RVO16(8, 2, 2, 3 | 768),        RVO16(4, 2, 2, 3 | 256),        RVO16(4, 2, 2, 3),
             RVO16(4, 3, 2, 3 | 768 | 4096), RVO16(8, 2, 2, 3 | 768 | 4096)};
    if (getenv("RANGES_R3C")) // round 3: CH2 against CH4 / CH8 by value span
        V = {RVO16(2, 2, 2, 3 | 768), RVO16(4, 2, 2, 3 | 768), RVO16(8, 2, 2, 3 | 768)};
    if (getenv("RANGES_R3D")) // round 3: the per-wave chunk size (OPT bit 14) against fixed CH2 / CH4 / CH8
        V = {RVO16(2, 2, 2, 3 | 768), RVO16(2, 2, 2, 3 | 768 | 16384), RVO16(4, 2, 2, 3 | 768),
             RVO16(8, 2, 2, 3 | 768)};
    if (getenv("RANGES_R3E")) // round 3: the per-wave chunk size in the two 8-wave workgroups shape
        V = {RVO(2, 2, 2, 2, 3), RVO(2, 2, 2, 2, 3 | 16384), RVO(4, 2, 2, 2, 3), RVO(8, 2, 2, 2, 3)};
    if (getenv("RANGES_ALL")) // the earlier CH / NBUF / fold sweep
        V = {RV(2, 2, 2, 2),     RVO(2, 2, 2, 2, 1), RVO(2, 2, 2, 2, 2), RVO(2, 2, 2, 2, 3),
             RVO(1, 4, 2, 2, 3), RVO(2, 3, 2, 2, 3), RVO(4, 2, 2, 2, 3)};
    uint64_t nmax = 0;
    for (auto &s : sets)
        nmax = std::max(nmax, s.n);
    uint32_t *d_out, *d_ref;
    CK(hipMalloc(&d_out, nmax * 4));
    CK(hipMalloc(&d_ref, nmax * 4));
    CK(hipDeviceSynchronize());

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 5;
    bool ok_all = true;
    for (auto &s : sets) {
        std::vector<std::vector<float>> ms(V.size());
        for (int r = 0; r < rounds + 1; r++) {
            for (size_t vi = 0; vi < V.size(); vi++) {
                const uint64_t want = (s.n + kWaves - 1) / kWaves;
                const uint32_t grid = (uint32_t)std::min<uint64_t>(want, (uint64_t)ncu * V[vi].wg_per_cu);
                CK(hipEventRecord(e0, 0));
                if (r == 0)
                    CK(hipMemset(d_out, 0xA5, s.n * 4));
                for (int it = 0; it < iters; it++)
                    V[vi].launch(dim3(grid), d, s.n, s.d_off, s.d_len, s.stride, s.len_const,
                                 V[vi].g32 ? d_img32 : d_img, V[vi].g32 ? d_fold32 : d_fold, d_un, d_out);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (r > 0)
                    ms[vi].push_back(t / iters);
                if (r == 0) {
                    if (vi == 0)
                        CK(hipMemcpy(d_ref, d_out, s.n * 4, hipMemcpyDeviceToDevice));
                    else {
                        std::vector<uint32_t> a(s.n), b(s.n);
                        CK(hipMemcpy(a.data(), d_ref, s.n * 4, hipMemcpyDeviceToHost));
                        CK(hipMemcpy(b.data(), d_out, s.n * 4, hipMemcpyDeviceToHost));
                        if (!strstr(V[vi].name, "4096") && memcmp(a.data(), b.data(), s.n * 4)) { // 4096: roof
                            printf("MISMATCH %s %s\n", s.name, V[vi].name);
                            ok_all = false;
                        }
                    }
                }
            }
        }
        printf("== %s: %llu extents, %.2f GiB of values\n", s.name, (unsigned long long)s.n, s.bytes / (1 << 30));
        for (size_t vi = 0; vi < V.size(); vi++) {
            std::sort(ms[vi].begin(), ms[vi].end());
            const double med = ms[vi][ms[vi].size() / 2];
            printf("  %-32s median %8.4f ms  %7.1f GB/s  (best %7.1f)\n", V[vi].name, med, s.bytes / med / 1e6,
                   s.bytes / ms[vi][0] / 1e6);
        }
    }
    printf("variants bit-identical: %s\n", ok_all ? "yes" : "NO");
    return ok_all ? 0 : 1;
}
