// Streaming job queue for block script checks.
// Parity: reference src/checkqueue.h:27-164 (CCheckQueue: a master thread pushes CScriptCheck
// batches while N-1 workers drain them; the master joins the work in Wait()) and
// src/validation.cpp:1740-1745 (ThreadScriptCheck). Differences in this design:
//  * jobs are published as a growing prefix [0, avail) of a caller-owned array (no copies into
//    a shared vector), claimed in adaptive batches under one mutex;
//  * idle workers sleep on a condition variable (never spin), so a block's UTXO pass keeps
//    its core while the queue is empty;
//  * the queue owns its threads: it is independent of WorkerPool, so pool users (sighash
//    midstates, the GPU batch prep) are never blocked by an open session, and a job function
//    may itself use a WorkerPool;
//  * the result is not reduced here: the job function records failures (the ECDSA work
//    itself is deferred to the batch verifier, csrc/node/sigverify.h).
#pragma once
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bcp {

class CheckQueue {
public:
    // nWorkers threads besides the caller (0: everything runs on the caller in Complete()).
    explicit CheckQueue(int nWorkers);
    ~CheckQueue();
    CheckQueue(const CheckQueue&) = delete;
    CheckQueue& operator=(const CheckQueue&) = delete;

    // Opens a session: fn(k) is run for every published job index k. One session at a time.
    void Begin(std::function<void(size_t)> fn);
    // Jobs [0, total) are now available (total never decreases within a session).
    void Publish(size_t total);
    // No more jobs: the caller runs jobs too until all published ones are done, then the
    // session closes. Safe to call on an unopened session (no-op).
    void Complete();
    int Workers() const { return (int)threads.size(); }
    // Jobs executed by worker threads / by the completing caller since construction.
    size_t WorkerJobs() const;

private:
    void Loop();
    bool ClaimLocked(size_t& b, size_t& e);
    void WakeLocked();
    std::vector<std::thread> threads;
    mutable std::mutex m;
    std::condition_variable cvWork, cvDone;
    std::mutex sessionMutex;      // one open session per queue: held from Begin to Complete
    std::thread::id sessionOwner; // the thread that opened the session (guarded by m)
    std::function<void(size_t)> fn;
    size_t avail = 0, next = 0, done = 0;
    size_t workerJobs = 0;
    size_t sleeping = 0; // workers waiting on cvWork
    bool active = false, stop = false;
};

} // namespace bcp
