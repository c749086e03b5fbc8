// queue_slots.h — ownership of the LDS pool kernels' work queues (pt_trace.hip).
//
// trace_pool_lds_kernel takes its (tile, chunk) items from a device-wide counter pair {next item, waves
// exited} in device memory.  Until round 5 a launch took the pair `g_next_queue++ % kPoolQueues` of a
// ring: a later launch could take a pair whose launch was still running (1024 LDS launches issued while
// one render is in flight — concurrent renders of other scenes, rt_hip.h), and both launches would then
// deal items from one counter: duplicated or skipped items, a reset in mid-flight, wrong sums and no
// error.  QueueSlots hands a pair out only while nobody holds it: a slot is held from acquire() until its
// release token (an event recorded on the launch's stream after the launch, and again after a cancel's
// clear kernel on that stream) has completed.  Host-only code: tests/test_queue_slots.py drives it from
// many threads with simulated tokens (tests/hostcheck/queue_slots_check.cpp).
#pragma once
#include <vector>

namespace rt {

// Token: the release token type (hipEvent_t in the library; the test's simulated completion flags).
// Not thread-safe by itself: the caller serializes every call with one lock (pt_trace.hip: g_launch_mu),
// which also covers the check-then-act of cancel_pool_launches on a held slot.
template <class Token>
class QueueSlots {
public:
    explicit QueueSlots(int n) : state_(n, kFree), tok_(n), gen_(n, 0) {}
    int size() const { return (int)state_.size(); }

    // A slot nobody holds — never used, released, or held by a token that done(token) reports complete —
    // now pending for the caller (no other acquire() takes it); -1 when every slot is pending or held by
    // an incomplete token.  The search starts after the last slot handed out, so slots rotate.
    template <class Done>
    int acquire(Done&& done) {
        const int n = size();
        for (int i = 0; i < n; ++i) {
            const int k = (cursor_ + i) % n;
            if (state_[k] == kPending) continue;
            if (state_[k] == kHeld && !done(tok_[k])) continue;
            state_[k] = kPending;
            ++gen_[k];
            cursor_ = (k + 1) % n;
            return k;
        }
        return -1;
    }
    // pending slot k is held until `release` completes (the launch was enqueued)
    void hold(int k, const Token& release) {
        tok_[k] = release;
        state_[k] = kHeld;
    }
    // pending slot k is free again (its launch was never enqueued)
    void abandon(int k) { state_[k] = kFree; }
    // held slot k: its release moved to a later token (a cancel's clear kernel after the launch)
    void extend(int k, const Token& release) {
        if (state_[k] == kHeld) tok_[k] = release;
    }
    bool held(int k) const { return state_[k] != kFree; }
    // generation of slot k: counts its acquisitions (a record of a launch on slot k is stale once it changed)
    unsigned generation(int k) const { return gen_[k]; }
    // the token slot k was last held with (the library keeps one event per slot and re-records it)
    Token& token(int k) { return tok_[k]; }

private:
    enum : unsigned char { kFree, kPending, kHeld };
    std::vector<unsigned char> state_;
    std::vector<Token> tok_;
    std::vector<unsigned> gen_;
    int cursor_ = 0;
};

}  // namespace rt
