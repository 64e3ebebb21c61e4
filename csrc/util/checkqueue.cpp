#include "util/checkqueue.h"

#include <algorithm>

namespace bcp {

// Largest batch one claim takes (reference checkqueue.h: nBatchSize 128 per script check; jobs
// here are script evaluations with deferred signatures, a few microseconds each).
static const size_t MAX_CLAIM = 16;
// Jobs per woken worker (a worker that finds more than it claimed wakes the next one).
static const size_t MIN_WAKE_JOBS = 4;

CheckQueue::CheckQueue(int nWorkers) {
    for (int i = 0; i < nWorkers; i++) threads.emplace_back([this] { Loop(); });
}

CheckQueue::~CheckQueue() {
    {
        std::lock_guard<std::mutex> l(m);
        stop = true;
    }
    cvWork.notify_all();
    for (auto& t : threads) t.join();
}

size_t CheckQueue::WorkerJobs() const {
    std::lock_guard<std::mutex> l(m);
    return workerJobs;
}

// Claims [b, e) of the published jobs: about an even share per thread, at most MAX_CLAIM.
bool CheckQueue::ClaimLocked(size_t& b, size_t& e) {
    if (!active || next >= avail) return false;
    const size_t left = avail - next;
    const size_t share = std::max<size_t>(1, std::min(MAX_CLAIM, left / (threads.size() + 1)));
    b = next;
    e = next + share;
    next = e;
    return true;
}

// Wakes as many sleeping workers as the unclaimed jobs can keep busy (called with m held). A
// notify_all per published transaction would wake every worker for two jobs: on a 21,000-tx
// block that is hundreds of thousands of futile wake-ups contending for m.
void CheckQueue::WakeLocked() {
    if (!active || next >= avail || sleeping == 0) return;
    const size_t want = std::min<size_t>(sleeping, (avail - next + MIN_WAKE_JOBS - 1) / MIN_WAKE_JOBS);
    for (size_t i = 0; i < want; i++) cvWork.notify_one();
}

void CheckQueue::Loop() {
    std::unique_lock<std::mutex> l(m);
    for (;;) {
        size_t b = 0, e = 0;
        ++sleeping;
        cvWork.wait(l, [&] { return stop || ClaimLocked(b, e); });
        --sleeping;
        if (stop) return;
        for (;;) {
            WakeLocked(); // more left than this claim: pass the work on (cascade)
            const std::function<void(size_t)>* f = &fn;
            l.unlock();
            for (size_t k = b; k < e; k++) (*f)(k);
            l.lock();
            done += e - b;
            workerJobs += e - b;
            if (done == avail) cvDone.notify_all();
            if (!ClaimLocked(b, e)) break; // keep going while there is work, without sleeping
        }
    }
}

void CheckQueue::Begin(std::function<void(size_t)> f) {
    sessionMutex.lock(); // a second caller blocks here until the open session completes
    std::lock_guard<std::mutex> l(m);
    fn = std::move(f);
    avail = next = done = 0;
    active = true;
    sessionOwner = std::this_thread::get_id();
}

void CheckQueue::Publish(size_t total) {
    std::lock_guard<std::mutex> l(m);
    if (!active || total <= avail) return;
    avail = total;
    WakeLocked();
}

void CheckQueue::Complete() {
    std::unique_lock<std::mutex> l(m);
    if (!active || sessionOwner != std::this_thread::get_id()) return; // no session of this thread
    size_t b = 0, e = 0;
    while (ClaimLocked(b, e)) { // the caller helps drain the queue
        l.unlock();
        for (size_t k = b; k < e; k++) fn(k);
        l.lock();
        done += e - b;
    }
    cvDone.wait(l, [&] { return done == avail; });
    active = false;
    sessionOwner = std::thread::id();
    fn = nullptr;
    avail = next = done = 0;
    l.unlock();
    sessionMutex.unlock();
}

} // namespace bcp
