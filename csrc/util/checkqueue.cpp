#include "util/checkqueue.h"

#include <algorithm>

namespace bcp {

// Largest batch one claim takes (reference checkqueue.h: nBatchSize 128 per script check; jobs
// here are script evaluations with deferred signatures, a few microseconds each).
static const size_t MAX_CLAIM = 16;

CheckQueue::CheckQueue(int nWorkers) : sessionLock(sessionMutex, std::defer_lock) {
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

void CheckQueue::Loop() {
    std::unique_lock<std::mutex> l(m);
    for (;;) {
        size_t b = 0, e = 0;
        cvWork.wait(l, [&] { return stop || ClaimLocked(b, e); });
        if (stop) return;
        const std::function<void(size_t)>* f = &fn;
        l.unlock();
        for (size_t k = b; k < e; k++) (*f)(k);
        l.lock();
        done += e - b;
        workerJobs += e - b;
        if (done == avail) cvDone.notify_all();
    }
}

void CheckQueue::Begin(std::function<void(size_t)> f) {
    sessionLock.lock();
    std::lock_guard<std::mutex> l(m);
    fn = std::move(f);
    avail = next = done = 0;
    active = true;
}

void CheckQueue::Publish(size_t total) {
    {
        std::lock_guard<std::mutex> l(m);
        if (!active || total <= avail) return;
        avail = total;
    }
    cvWork.notify_all();
}

void CheckQueue::Complete() {
    if (!sessionLock.owns_lock()) return;
    std::unique_lock<std::mutex> l(m);
    size_t b = 0, e = 0;
    while (ClaimLocked(b, e)) { // the caller helps drain the queue
        l.unlock();
        for (size_t k = b; k < e; k++) fn(k);
        l.lock();
        done += e - b;
    }
    cvDone.wait(l, [&] { return done == avail; });
    active = false;
    fn = nullptr;
    avail = next = done = 0;
    l.unlock();
    sessionLock.unlock();
}

} // namespace bcp
