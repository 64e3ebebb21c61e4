// Mutex wrapper with lock-order (potential deadlock) detection.
// Parity: reference src/sync.{h,cpp} (CCriticalSection = AnnotatedMixin<recursive_mutex>,
// DEBUG_LOCKORDER: per-thread lock stacks, global map of observed lock pairs,
// potential_deadlock_detected() reporting both orders, AssertLockHeld/AssertLockNotHeld).
//
// Design: the check is compiled in always and switched on at run time
// (-debuglockorder, or SetLockOrderChecking(true) in tests); when off, lock()/unlock()
// cost one relaxed atomic load.
#pragma once
#include "util/threadsafety.h"

#include <atomic>
#include <mutex>
#include <string>

namespace bcp {

void SetLockOrderChecking(bool on, bool abortOnDeadlock = true);
bool LockOrderChecking();
// Number of potential deadlocks reported so far (tests).
uint64_t LockOrderViolations();

namespace detail {
extern std::atomic<bool> g_lockorder;
void EnterCritical(const void* cs, const char* name);
void LeaveCritical(const void* cs);
bool HoldsLock(const void* cs);
} // namespace detail

class CAPABILITY("mutex") CCriticalSection : public std::recursive_mutex {
public:
    explicit CCriticalSection(const char* name = "cs") : name(name) {}
    void lock() ACQUIRE() {
        if (detail::g_lockorder.load(std::memory_order_relaxed)) detail::EnterCritical(this, name);
        std::recursive_mutex::lock();
    }
    void unlock() RELEASE() {
        std::recursive_mutex::unlock();
        if (detail::g_lockorder.load(std::memory_order_relaxed)) detail::LeaveCritical(this);
    }
    bool try_lock() TRY_ACQUIRE(true) {
        if (!std::recursive_mutex::try_lock()) return false;
        if (detail::g_lockorder.load(std::memory_order_relaxed)) detail::EnterCritical(this, name);
        return true;
    }
    const char* Name() const { return name; }

private:
    const char* name;
};

// A plain (non-recursive) std::mutex the thread-safety analysis can see: for members guarded by a
// leaf lock that is never waited on with a condition variable.
class CAPABILITY("mutex") Mutex : public std::mutex {
public:
    void lock() ACQUIRE() { std::mutex::lock(); }
    void unlock() RELEASE() { std::mutex::unlock(); }
    bool try_lock() TRY_ACQUIRE(true) { return std::mutex::try_lock(); }
};

// Only meaningful while lock-order checking is on.
void AssertLockHeldImpl(const CCriticalSection& cs, const char* file, int line) ASSERT_EXCLUSIVE_LOCK(cs);
void AssertLockNotHeldImpl(const CCriticalSection& cs, const char* file, int line);
#define AssertLockHeld(cs) ::bcp::AssertLockHeldImpl(cs, __FILE__, __LINE__)
#define AssertLockNotHeld(cs) ::bcp::AssertLockNotHeldImpl(cs, __FILE__, __LINE__)

} // namespace bcp

// std::lock_guard over a CCriticalSection as a scoped capability, so the 200-odd
// `std::lock_guard<CCriticalSection> l(cs);` scopes are visible to the thread-safety analysis
// (a specialisation for a program-defined type; behaviour is the primary template's).
namespace std {
template <> class SCOPED_CAPABILITY lock_guard<bcp::CCriticalSection> {
public:
    explicit lock_guard(bcp::CCriticalSection& m) ACQUIRE(m) : m(m) { m.lock(); }
    lock_guard(bcp::CCriticalSection& m, adopt_lock_t) ACQUIRE(m) : m(m) {}
    ~lock_guard() RELEASE() { m.unlock(); }
    lock_guard(const lock_guard&) = delete;
    lock_guard& operator=(const lock_guard&) = delete;

private:
    bcp::CCriticalSection& m;
};
template <> class SCOPED_CAPABILITY lock_guard<bcp::Mutex> {
public:
    explicit lock_guard(bcp::Mutex& m) ACQUIRE(m) : m(m) { m.lock(); }
    ~lock_guard() RELEASE() { m.unlock(); }
    lock_guard(const lock_guard&) = delete;
    lock_guard& operator=(const lock_guard&) = delete;

private:
    bcp::Mutex& m;
};
} // namespace std
