// Deferred destruction: a block's connect leaves ~150k heap objects behind (script-job sinks,
// per-transaction sighash midstates, undo records, the per-block coins view). Freeing them is
// 10-17 ms of pointer chasing on the connecting thread; handing them to this thread instead lets
// the next block start while they are freed on another core. The queue is bounded, so a caller
// that outruns the reaper waits for it rather than piling up memory.
#pragma once
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

namespace bcp {

class Reaper {
public:
    static Reaper& Get();

    // take ownership of `v` and destroy it on the reaper thread
    template <typename T> void Drop(T&& v) {
        Push(std::unique_ptr<Base>(new Holder<std::decay_t<T>>(std::forward<T>(v))));
    }
    // wait until everything dropped so far is destroyed
    void Drain();

    ~Reaper();

private:
    struct Base {
        virtual ~Base() = default;
    };
    template <typename T> struct Holder : Base {
        explicit Holder(T&& x) : v(std::move(x)) {}
        T v;
    };
    static constexpr size_t MAX_PENDING = 32;

    Reaper();
    void Push(std::unique_ptr<Base> p);
    void Run();

    std::mutex mu;
    std::condition_variable cv, cvSpace;
    std::deque<std::unique_ptr<Base>> q;
    size_t busy = 0;
    bool stop = false;
    std::thread worker;
};

} // namespace bcp
