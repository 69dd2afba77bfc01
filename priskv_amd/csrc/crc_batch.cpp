// crc_batch.cpp -- SET-completion CRC batcher (include/priskv_crc_gpu.h).
//
// PrisKV completes a SET when the RDMA READ of the value into its block has
// landed (server/rdma.c:1417-1418 -> server/kv.c:505), one request at a time
// on each io thread.  A GPU launch per value would cost more than the value's
// CRC, so completions are queued here and hashed in batches: io threads call
// priskv_crc_batch_submit[v](value_off, valuelen, cookie), a worker thread
// takes the queue when it holds max_batch values or its oldest value has
// waited max_delay_us, runs ONE zero-copy extents pass over the registered
// value region (priskv_crc32_ranges_host) per max_batch values, and calls
// back (cookie, crc, status) for each value.  Built only on the public C ABI.
//
// Submission is sharded: each submitting thread keeps one shard (its own lock,
// so 16 io threads do not serialise on one mutex) and the shards share only an
// atomic count of queued values; the worker is woken on the empty -> non-empty
// transition and when the count reaches max_batch.  Callbacks for one thread's
// submissions come in that thread's submission order.
//
// Flush is by gather generation, not by counts: the worker numbers each pass
// over the shards (gen_started, under mu) and publishes the number of the last
// pass whose callbacks are done (gen_done).  A value whose submit returned
// before flush() read gen_started is in a shard before pass gen_started + 1
// visits that shard, so it is called back by the time gen_done reaches
// gen_started + 1.  (Counting values instead is racy: a pass visits the shards
// one by one and can pick up a later value from one shard while an earlier
// value in a shard it already visited waits for the next pass.)
#include <errno.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/priskv_crc_gpu.h"

namespace {
using Clock = std::chrono::steady_clock;
constexpr uint64_t kBacklogBatches = 8; // submitters wait beyond 8 * max_batch queued values
constexpr unsigned kShards = 32;

struct Shard {
    std::mutex mu;
    std::vector<uint64_t> off, cookie;
    std::vector<uint32_t> len;
    char pad[64];
};

unsigned my_shard()
{
    static std::atomic<unsigned> next{0};
    thread_local unsigned s = next.fetch_add(1, std::memory_order_relaxed) % kShards;
    return s;
}

int64_t now_ns() { return Clock::now().time_since_epoch().count(); }
} // namespace

struct priskv_crc_batch {
    priskv_crc_ctx *ctx = nullptr;
    const uint8_t *region = nullptr;
    uint64_t region_bytes = 0;
    bool registered_here = false;
    uint32_t max_batch = 0;
    int64_t max_delay_ns = 0;
    priskv_crc_batch_cb cb = nullptr;
    void *arg = nullptr;

    Shard shards[kShards];
    std::atomic<uint64_t> queued{0};     // values in the shards
    std::atomic<int64_t> oldest_ns{0};   // when the queue last became non-empty
    std::mutex mu;                       // worker sleep / flush / backpressure
    std::condition_variable cv_work, cv_room, cv_done;
    uint64_t gen_started = 0;            // guarded by mu: passes over the shards begun
    uint64_t gen_done = 0;               // guarded by mu: passes whose callbacks are done
    uint64_t flush_target = 0;           // guarded by mu: a flusher waits for gen_done >= this
    // set by destroy, which by contract runs with no submit in flight; read
    // by submitters without the lock (it only turns late misuse into -EINVAL)
    std::atomic<bool> stop{false};
    std::thread worker;

    void wake()
    {
        std::lock_guard<std::mutex> lk(mu);
        cv_work.notify_one();
    }

    // called by a submitter after it queued k values (prev = count before)
    void queued_more(uint64_t prev, uint64_t k)
    {
        if (prev == 0)
            oldest_ns.store(now_ns(), std::memory_order_relaxed);
        if (prev == 0 || (prev < max_batch && prev + k >= max_batch))
            wake();
        if (prev + k > kBacklogBatches * max_batch) {
            std::unique_lock<std::mutex> lk(mu);
            cv_room.wait(lk, [this] { return queued.load() <= kBacklogBatches * max_batch || stop.load(); });
        }
    }

    void run()
    {
        std::vector<uint64_t> off, cookie;
        std::vector<uint32_t> len, crc;
        for (;;) {
            uint64_t gen;
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    const uint64_t q = queued.load();
                    if (q >= max_batch || (stop.load() && q) || gen_done < flush_target)
                        break; // a flusher's pass runs even when nothing is queued
                    if (q == 0) {
                        if (stop.load())
                            return;
                        cv_work.wait(lk);
                        continue;
                    }
                    const auto deadline =
                        Clock::time_point(Clock::duration(oldest_ns.load(std::memory_order_relaxed) + max_delay_ns));
                    if (cv_work.wait_until(lk, deadline) == std::cv_status::timeout)
                        break;
                }
                gen = ++gen_started;
            }
            off.clear();
            len.clear();
            cookie.clear();
            for (Shard &s : shards) {
                std::lock_guard<std::mutex> lk(s.mu);
                off.insert(off.end(), s.off.begin(), s.off.end());
                len.insert(len.end(), s.len.begin(), s.len.end());
                cookie.insert(cookie.end(), s.cookie.begin(), s.cookie.end());
                s.off.clear();
                s.len.clear();
                s.cookie.clear();
            }
            if (queued.fetch_sub(off.size()) != off.size())
                oldest_ns.store(now_ns(), std::memory_order_relaxed); // values left: their age restarts
            {
                std::lock_guard<std::mutex> lk(mu);
                cv_room.notify_all();
            }
            crc.assign(off.size(), 0);
            for (size_t b = 0; b < off.size(); b += max_batch) {
                const size_t n = off.size() - b < max_batch ? off.size() - b : max_batch;
                const int rc = priskv_crc32_ranges_host(ctx, region, region_bytes, off.data() + b, len.data() + b,
                                                        n, crc.data() + b);
                for (size_t i = b; i < b + n; i++)
                    cb(arg, cookie[i], crc[i], rc);
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                gen_done = gen;
            }
            cv_done.notify_all();
        }
    }
};

// built with -fvisibility=hidden: only the C ABI leaves the library
#define PRV_API __attribute__((visibility("default")))

extern "C" {

PRV_API int priskv_crc_batch_create(priskv_crc_ctx *ctx, const void *h_region, uint64_t region_bytes,
                                    uint32_t max_batch, uint32_t max_delay_us, priskv_crc_batch_cb cb, void *arg,
                                    priskv_crc_batch **out)
{
    if (!ctx || !h_region || !region_bytes || !max_batch || !cb || !out)
        return -EINVAL;
    priskv_crc_batch *b = new (std::nothrow) priskv_crc_batch;
    if (!b)
        return -ENOMEM;
    b->ctx = ctx;
    b->region = (const uint8_t *)h_region;
    b->region_bytes = region_bytes;
    b->max_batch = max_batch;
    b->max_delay_ns = (int64_t)max_delay_us * 1000;
    b->cb = cb;
    b->arg = arg;
    // pin + map the value region once (already registered: use as is)
    const int rc = priskv_crc_host_register((void *)h_region, region_bytes);
    if (rc == 0)
        b->registered_here = true;
    else if (rc != -EEXIST) {
        delete b;
        return rc;
    }
    try {
        b->worker = std::thread([b] { b->run(); });
    } catch (...) {
        if (b->registered_here)
            priskv_crc_host_unregister((void *)h_region);
        delete b;
        return -ENOMEM;
    }
    *out = b;
    return 0;
}

PRV_API int priskv_crc_batch_submitv(priskv_crc_batch *b, uint64_t n, const uint64_t *value_offs,
                                     const uint32_t *valuelens, const uint64_t *cookies)
{
    if (!b || (n && (!value_offs || !valuelens || !cookies)))
        return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (value_offs[i] > b->region_bytes || valuelens[i] > b->region_bytes - value_offs[i])
            return -EINVAL;
    if (n == 0)
        return 0;
    if (b->stop.load(std::memory_order_relaxed))
        return -EINVAL;
    // count first, then publish: `queued` never drops below the values in the
    // shards, so the worker's subtraction of what it gathered cannot wrap
    const uint64_t prev = b->queued.fetch_add(n);
    Shard &s = b->shards[my_shard()];
    {
        std::lock_guard<std::mutex> lk(s.mu);
        s.off.insert(s.off.end(), value_offs, value_offs + n);
        s.len.insert(s.len.end(), valuelens, valuelens + n);
        s.cookie.insert(s.cookie.end(), cookies, cookies + n);
    }
    b->queued_more(prev, n);
    return 0;
}

PRV_API int priskv_crc_batch_submit(priskv_crc_batch *b, uint64_t value_off, uint32_t valuelen, uint64_t cookie)
{
    return priskv_crc_batch_submitv(b, 1, &value_off, &valuelen, &cookie);
}

PRV_API int priskv_crc_batch_flush(priskv_crc_batch *b)
{
    if (!b)
        return -EINVAL;
    std::unique_lock<std::mutex> lk(b->mu);
    // the first pass to begin after this point sees every value published
    // before it (see the file comment)
    const uint64_t target = b->gen_started + 1;
    if (b->flush_target < target)
        b->flush_target = target;
    b->cv_work.notify_one();
    b->cv_done.wait(lk, [b, target] { return b->gen_done >= target; });
    return 0;
}

PRV_API void priskv_crc_batch_destroy(priskv_crc_batch *b)
{
    if (!b)
        return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop.store(true); // the worker drains the queue, then exits
        b->cv_work.notify_one();
        b->cv_room.notify_all();
    }
    if (b->worker.joinable())
        b->worker.join();
    if (b->registered_here)
        priskv_crc_host_unregister((void *)b->region);
    delete b;
}

} // extern "C"
