// queue_slots_check.cpp — TEST INFRASTRUCTURE: drives rt::QueueSlots (blenderraytracer_amd/csrc/
// queue_slots.h, the LDS pool launches' queue ownership) from many threads with simulated release
// tokens, and counts every slot handed out while another launch still held it.
//
// A "launch" acquires a slot, marks itself its owner, holds the slot with a token (a completion flag a
// later step sets), and ends some iterations later: it clears its ownership first, then completes its
// token.  Some launches are "cancelled": their release is extended to a second token (the clear kernel
// after the move) that completes later still, and their ownership lasts until then.  Some acquisitions
// are abandoned (the launch failed to enqueue).  A correct allocator never hands out a slot whose owner
// is set.  `broken` replaces the completion test with one that always says "done" (the round-5 ring's
// behaviour): the checker must then see violations.
//
// usage: queue_slots_check <threads> <launches per thread> <slots> <broken 0|1>
// prints: violations=<n> acquired=<n> waits=<n> extended=<n> abandoned=<n>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../blenderraytracer_amd/csrc/queue_slots.h"

using Flag = std::shared_ptr<std::atomic<bool>>;

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    const int launches = argc > 2 ? atoi(argv[2]) : 20000;
    const int nslots = argc > 3 ? atoi(argv[3]) : 16;
    const bool broken = argc > 4 && atoi(argv[4]) != 0;

    rt::QueueSlots<Flag> slots(nslots);
    std::mutex mu;                                   // the library's g_launch_mu
    std::vector<std::atomic<int>> owner(nslots);
    for (auto& o : owner) o.store(-1);
    std::atomic<long long> violations{0}, acquired{0}, waits{0}, extended{0}, abandoned{0};

    // single-threaded properties first: exhaustion, rotation, generations, abandon
    {
        rt::QueueSlots<Flag> s(4);
        auto done = [](const Flag& f) { return !f || f->load(); };
        std::vector<int> got;
        for (int i = 0; i < 4; ++i) got.push_back(s.acquire(done));
        if (s.acquire(done) != -1) ++violations;     // all pending: none left
        for (int i = 0; i < 4; ++i)
            if (got[i] != i || s.generation(i) != 1u) ++violations;
        s.abandon(2);
        if (s.acquire(done) != 2 || s.generation(2) != 2u) ++violations;
        Flag f = std::make_shared<std::atomic<bool>>(false);
        s.hold(0, f);
        s.abandon(1);
        s.abandon(2);
        s.abandon(3);
        if (s.acquire(done) != 3) ++violations;       // rotation: the search starts after the last handed out (2)
        // 0 is held by an incomplete token: never handed out
        for (int i = 0; i < 8; ++i) {
            const int k = s.acquire(done);
            if (k == 0) ++violations;
            if (k >= 0) s.abandon(k);
        }
        f->store(true);
        bool seen0 = false;
        for (int i = 0; i < 4; ++i) {
            const int k = s.acquire(done);
            seen0 = seen0 || k == 0;
            if (k >= 0) s.abandon(k);
        }
        if (!seen0) ++violations;
    }

    auto worker = [&](int id) {
        std::mt19937 rng(1234u + 7u * (unsigned)id);
        struct Launch { int slot, end_at; Flag first, second; };
        std::deque<Launch> inflight;
        auto done = [&](const Flag& f) { return broken || !f || f->load(); };
        auto finish = [&](Launch& l) {
            // the launch (and, for a cancelled one, its clear) ends: ownership first, then the token(s)
            int me = id;
            if (!owner[l.slot].compare_exchange_strong(me, -1)) ++violations;
            l.first->store(true);
            if (l.second) l.second->store(true);
        };
        for (int it = 0; it < launches; ++it) {
            // retire the launches whose time has come (FIFO per thread, like one stream)
            while (!inflight.empty() && (inflight.front().end_at <= it || inflight.size() > 6)) {
                finish(inflight.front());
                inflight.pop_front();
            }
            int k;
            for (;;) {
                {
                    std::lock_guard<std::mutex> g(mu);
                    k = slots.acquire(done);
                }
                if (k >= 0) break;
                ++waits;
                if (!inflight.empty()) {              // nothing free: our own oldest launch ends
                    finish(inflight.front());
                    inflight.pop_front();
                } else {
                    std::this_thread::yield();
                }
            }
            int none = -1;
            if (!owner[k].compare_exchange_strong(none, id)) {
                ++violations;                         // handed out while another launch holds it
                std::lock_guard<std::mutex> g(mu);    // (broken mode: give it back, keep going)
                slots.abandon(k);
                continue;
            }
            ++acquired;
            const unsigned r = rng();
            if (r % 17 == 0) {                        // failed to enqueue: the slot goes back at once
                owner[k].store(-1);
                std::lock_guard<std::mutex> g(mu);
                slots.abandon(k);
                ++abandoned;
                continue;
            }
            Launch l{k, it + 1 + (int)(r % 5), std::make_shared<std::atomic<bool>>(false), nullptr};
            {
                std::lock_guard<std::mutex> g(mu);
                slots.hold(k, l.first);
            }
            if ((r >> 8) % 5 == 0) {                  // cancelled: the release moves to the clear's token
                l.second = std::make_shared<std::atomic<bool>>(false);
                std::lock_guard<std::mutex> g(mu);
                slots.extend(k, l.second);
                ++extended;
            }
            // the launch's first token may complete before the clear's (the launch ended, the clear
            // has not run): the slot must stay held
            if (l.second && (r >> 12) % 2 == 0) l.first->store(true);
            inflight.push_back(l);
        }
        while (!inflight.empty()) {
            finish(inflight.front());
            inflight.pop_front();
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t);
    for (auto& t : pool) t.join();
    printf("violations=%lld acquired=%lld waits=%lld extended=%lld abandoned=%lld\n", violations.load(),
           acquired.load(), waits.load(), extended.load(), abandoned.load());
    return 0;
}
