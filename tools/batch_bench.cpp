// batch_bench.cpp -- SET-completion batcher under io-thread load (tool, not product).
//
// T submitter threads play PrisKV io threads completing SETs (server/rdma.c:1417
// -> server/kv.c:505): each submits (value_off, valuelen) of a ~value_size value
// at a random block of a host value region (anonymous mmap, registered by the
// batcher), as fast as it can, for `secs` seconds.  Reports values/s, GiB/s and
// the submit -> callback latency percentiles per (max_batch, max_delay_us), and
// the same T threads hashing the same kind of values on the CPU with the host
// priskv_crc32 (include/crc.h) for comparison.  A 1/256 sample of the callback
// CRCs is checked against priskv_crc32.
// usage: batch_bench [region_GiB=4] [value_size=4096] [threads=16] [secs=2] [per_call=1]
// (per_call > 1: submitters use priskv_crc_batch_submitv with that many values)
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../include/crc.h"
#include "../include/priskv_crc_gpu.h"

using Clock = std::chrono::steady_clock;

static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Shared {
    const uint8_t *region;
    uint64_t region_bytes;
    std::vector<std::vector<int64_t>> t_submit; // [thread][seq % cap] ns
    uint64_t cap;
    std::atomic<uint64_t> done{0}, bad{0}, checked{0}, errors{0};
    std::vector<std::atomic<uint64_t>> hist; // latency buckets of 1 us
    std::vector<uint64_t> off_of, len_of;    // per thread: last submitted (for the CRC sample)
    Shared() : hist(100000) {}
};

static int64_t now_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

static void on_crc(void *arg, uint64_t cookie, uint32_t crc, int status)
{
    Shared *s = (Shared *)arg;
    const uint64_t t = cookie >> 40, seq = cookie & ((1ull << 40) - 1);
    const int64_t lat = now_ns() - s->t_submit[t][seq % s->cap];
    const uint64_t us = (uint64_t)(lat / 1000);
    s->hist[us < s->hist.size() ? us : s->hist.size() - 1]++;
    if (status)
        s->errors++;
    if ((seq & 255) == 0) { // re-derive this value's extent and check its CRC
        uint64_t h = mix64(cookie);
        const uint64_t blocks = s->region_bytes / 4096 - 64;
        const uint64_t off = (h % blocks) * 4096;
        const uint32_t len = (uint32_t)(s->len_of[t] - (mix64(h) & 63));
        if (priskv_crc32((uint8_t *)s->region + off, len) != crc)
            s->bad++;
        s->checked++;
    }
    s->done++;
}

static double pct(const std::vector<std::atomic<uint64_t>> &h, uint64_t total, double q)
{
    uint64_t acc = 0, want = (uint64_t)(q * (double)total);
    for (size_t i = 0; i < h.size(); i++) {
        acc += h[i].load();
        if (acc > want)
            return (double)i;
    }
    return (double)h.size();
}

int main(int argc, char **argv)
{
    const uint64_t gib = argc > 1 ? strtoull(argv[1], 0, 0) : 4;
    const uint32_t vsize = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096;
    const int T = argc > 3 ? atoi(argv[3]) : 16;
    const double secs = argc > 4 ? atof(argv[4]) : 2.0;
    const uint32_t per_call = argc > 5 ? (uint32_t)atoi(argv[5]) : 1;
    const uint64_t bytes = gib << 30;
    uint8_t *region = (uint8_t *)mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (region == MAP_FAILED) {
        perror("mmap");
        return 1;
    }
    {
        std::vector<std::thread> f;
        for (int t = 0; t < 16; t++)
            f.emplace_back([=] {
                for (uint64_t i = (uint64_t)t; i < bytes / 8; i += 16)
                    ((uint64_t *)region)[i] = mix64(0x5EED5EEDull + i);
            });
        for (auto &x : f)
            x.join();
    }
    priskv_crc_ctx *ctx = nullptr;
    if (int rc = priskv_crc_ctx_create(0, &ctx)) {
        fprintf(stderr, "ctx_create: %d\n", rc);
        return 1;
    }
    const uint64_t blocks = bytes / 4096 - 64;

    // CPU comparison: the same T threads hashing values with priskv_crc32
    {
        std::atomic<uint64_t> n{0};
        std::vector<std::thread> th;
        const auto t0 = Clock::now();
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                uint64_t i = 0, sink = 0;
                while (std::chrono::duration<double>(Clock::now() - t0).count() < secs) {
                    const uint64_t h = mix64(((uint64_t)t << 40) | i++);
                    sink += priskv_crc32(region + (h % blocks) * 4096, vsize - (uint32_t)(mix64(h) & 63));
                }
                n += i + (sink == 42);
            });
        for (auto &x : th)
            x.join();
        const double el = std::chrono::duration<double>(Clock::now() - t0).count();
        printf("{\"path\": \"cpu_priskv_crc32\", \"threads\": %d, \"value_size\": %u, \"values_per_s\": %.0f, "
               "\"GiBs\": %.2f}\n",
               T, vsize, n / el, n * (double)vsize / el / (1 << 30));
        fflush(stdout);
    }

    const uint32_t batches[] = {256, 1024, 4096, 16384};
    for (uint32_t mb : batches) {
        Shared s;
        s.region = region;
        s.region_bytes = bytes;
        s.cap = 1 << 22;
        s.t_submit.assign(T, std::vector<int64_t>(s.cap));
        s.len_of.assign(T, vsize);
        priskv_crc_batch *b = nullptr;
        if (int rc = priskv_crc_batch_create(ctx, region, bytes, mb, 500, on_crc, &s, &b)) {
            fprintf(stderr, "batch_create: %d\n", rc);
            return 1;
        }
        std::atomic<uint64_t> submitted{0};
        std::vector<std::thread> th;
        const auto t0 = Clock::now();
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                uint64_t i = 0;
                std::vector<uint64_t> o(per_call), c(per_call);
                std::vector<uint32_t> l(per_call);
                while (std::chrono::duration<double>(Clock::now() - t0).count() < secs) {
                    const int64_t ts = now_ns();
                    for (uint32_t k = 0; k < per_call; k++) {
                        c[k] = ((uint64_t)t << 40) | (i + k);
                        const uint64_t h = mix64(c[k]);
                        o[k] = (h % blocks) * 4096;
                        l[k] = vsize - (uint32_t)(mix64(h) & 63);
                        s.t_submit[t][(i + k) % s.cap] = ts;
                    }
                    if (priskv_crc_batch_submitv(b, per_call, o.data(), l.data(), c.data()))
                        break;
                    i += per_call;
                }
                submitted += i;
            });
        for (auto &x : th)
            x.join();
        priskv_crc_batch_flush(b);
        const double el = std::chrono::duration<double>(Clock::now() - t0).count();
        priskv_crc_batch_destroy(b);
        const uint64_t n = s.done.load();
        printf("{\"path\": \"set_batcher\", \"threads\": %d, \"per_call\": %u, \"value_size\": %u, \"max_batch\": %u, "
               "\"max_delay_us\": 500, \"values\": %lu, \"values_per_s\": %.0f, \"GiBs\": %.2f, "
               "\"lat_us_p50\": %.0f, \"lat_us_p99\": %.0f, \"lat_us_max_bucket\": %.0f, \"checked\": %lu, "
               "\"bad\": %lu, \"errors\": %lu}\n",
               T, per_call, vsize, mb, (unsigned long)n, n / el, n * (double)vsize / el / (1 << 30), pct(s.hist, n, 0.5),
               pct(s.hist, n, 0.99), pct(s.hist, n, 0.99999), (unsigned long)s.checked.load(),
               (unsigned long)s.bad.load(), (unsigned long)s.errors.load());
        fflush(stdout);
        if (submitted.load() != n)
            printf("# submitted %lu != called back %lu\n", (unsigned long)submitted.load(), (unsigned long)n);
    }
    priskv_crc_ctx_destroy(ctx);
    munmap(region, bytes);
    return 0;
}
