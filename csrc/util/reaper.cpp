#include "util/reaper.h"

namespace bcp {

Reaper& Reaper::Get() {
    static Reaper r;
    return r;
}

Reaper::Reaper() : worker([this] { Run(); }) {}

Reaper::~Reaper() {
    {
        std::lock_guard<std::mutex> l(mu);
        stop = true;
    }
    cv.notify_all();
    worker.join(); // drains what is queued first
}

void Reaper::Push(std::unique_ptr<Base> p) {
    std::unique_lock<std::mutex> l(mu);
    cvSpace.wait(l, [&] { return q.size() < MAX_PENDING; });
    q.push_back(std::move(p));
    l.unlock();
    cv.notify_one();
}

void Reaper::Drain() {
    std::unique_lock<std::mutex> l(mu);
    cvSpace.wait(l, [&] { return q.empty() && busy == 0; });
}

void Reaper::Run() {
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
        cv.wait(l, [&] { return stop || !q.empty(); });
        if (q.empty()) return; // stop requested and nothing left
        std::unique_ptr<Base> p = std::move(q.front());
        q.pop_front();
        busy++;
        l.unlock();
        p.reset();
        l.lock();
        busy--;
        cvSpace.notify_all();
    }
}

} // namespace bcp
