// checkqueue_tests: the block script-check queue, the worker pool and the scheduler.
// Parity: reference src/test/scheduler_tests.cpp (manythreads: many tasks rescheduling each
// other, the counters balance) and, for the script-check queue, the properties the reference's
// CCheckQueue users rely on (src/validation.cpp:1740-1745, 2011-2127):
// * every queued job runs exactly once;
// * jobs published in pieces during the UTXO pass are all drained by Complete();
// * sessions are independent;
// * an empty session completes;
// * the queue works with no worker threads at all.
#include "test/unittest.h"

#include "util/checkqueue.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <atomic>
#include <chrono>
#include <thread>

using namespace bcp;

TEST_CASE(checkqueue_tests, every_job_once) {
    for (int workers : {0, 1, 3, 15}) {
        CheckQueue q(workers);
        FastRandomContext rng(true);
        for (int session = 0; session < 20; session++) {
            const size_t n = (size_t)rng.randrange(5000);
            std::vector<std::atomic<int>> hits(n);
            for (auto& h : hits) h = 0;
            q.Begin([&](size_t k) { hits[k].fetch_add(1, std::memory_order_relaxed); });
            // publish in random pieces, as the UTXO pass does, with some idle gaps
            size_t pub = 0;
            while (pub < n) {
                pub = std::min(n, pub + 1 + (size_t)rng.randrange(300));
                q.Publish(pub);
                if (rng.randrange(8) == 0) std::this_thread::yield();
            }
            q.Complete();
            size_t bad = 0;
            for (auto& h : hits) bad += h.load() != 1;
            if (bad) {
                test::RecordFailure(strprintf("%zu of %zu jobs not run exactly once (%d workers)", bad, n, workers),
                                    __FILE__, __LINE__);
                return;
            }
        }
        // an empty session and a Complete() without Begin() are no-ops
        q.Begin([](size_t) {});
        q.Complete();
        q.Complete();
    }
}

TEST_CASE(checkqueue_tests, complete_waits_for_running_jobs) {
    // jobs still running on workers when the caller runs out of claims must be waited for
    CheckQueue q(4);
    std::atomic<int> finished{0};
    q.Begin([&](size_t) {
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        finished++;
    });
    q.Publish(40);
    q.Complete();
    CHECK_EQ(finished.load(), 40);
    // a stale Publish after Complete does nothing
    q.Publish(100);
    CHECK_EQ(finished.load(), 40);
}

TEST_CASE(checkqueue_tests, workers_take_load) {
    // with slow jobs, the workers (not only the completing caller) execute most of them
    CheckQueue q(7);
    const size_t before = q.WorkerJobs();
    q.Begin([](size_t) { std::this_thread::sleep_for(std::chrono::microseconds(200)); });
    for (size_t k = 16; k <= 512; k += 16) q.Publish(k);
    q.Complete();
    CHECK(q.WorkerJobs() - before > 256u);
}

TEST_CASE(checkqueue_tests, worker_pool_parallel_for) {
    WorkerPool pool(8);
    for (size_t n : {0u, 1u, 7u, 64u, 1000u, 100003u}) {
        for (size_t grain : {1u, 16u, 1000u}) {
            std::vector<std::atomic<int>> hits(n);
            for (auto& h : hits) h = 0;
            pool.ParallelFor(n, [&](size_t i) { hits[i]++; }, grain);
            size_t bad = 0;
            for (auto& h : hits) bad += h.load() != 1;
            CHECK_EQ(bad, 0u);
        }
    }
    // calls from several threads serialise instead of interleaving
    std::atomic<int> inside{0}, maxInside{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; t++)
        ts.emplace_back([&] {
            for (int r = 0; r < 20; r++)
                pool.ParallelFor(64, [&](size_t) {
                    const int now = ++inside;
                    int m = maxInside.load();
                    while (now > m && !maxInside.compare_exchange_weak(m, now)) {}
                    --inside;
                }, 8);
        });
    for (auto& t : ts) t.join();
    CHECK(maxInside.load() <= pool.Size());
}

TEST_CASE(checkqueue_tests, scheduler_many_tasks) {
    // reference scheduler_tests manythreads: tasks that reschedule follow-up tasks; the
    // counters end at the number of initial tasks
    Scheduler sched;
    std::mutex mu;
    int counter[10] = {0};
    std::atomic<int> pending{0};
    FastRandomContext rng(true);
    for (int i = 0; i < 100; i++) {
        const int which = (int)rng.randrange(10), delta = (int)rng.randrange(2001) - 1000;
        const int64_t t1 = (int64_t)rng.randrange(20), t2 = 5 + (int64_t)rng.randrange(20);
        pending += 2;
        sched.ScheduleFromNow(
            [&, which, delta, t2] {
                {
                    std::lock_guard<std::mutex> l(mu);
                    counter[which] += delta;
                }
                sched.ScheduleFromNow(
                    [&, which, delta] {
                        std::lock_guard<std::mutex> l(mu);
                        counter[which] += 1 - delta;
                        pending--;
                    },
                    t2);
                pending--;
            },
            t1);
    }
    for (int i = 0; i < 500 && pending.load() > 0; i++) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    CHECK_EQ(pending.load(), 0);
    int sum = 0;
    {
        std::lock_guard<std::mutex> l(mu);
        for (int c : counter) sum += c;
    }
    CHECK_EQ(sum, 100);
    // a periodic task runs repeatedly until the scheduler stops
    std::atomic<int> ticks{0};
    sched.ScheduleEvery([&] { ticks++; }, 5);
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    sched.Stop();
    const int seen = ticks.load();
    CHECK(seen >= 3);
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    CHECK_EQ(ticks.load(), seen);
}
