// Mutex wrapper with lock-order (potential deadlock) detection.
// Parity: reference src/sync.{h,cpp} (CCriticalSection = AnnotatedMixin<recursive_mutex>,
// DEBUG_LOCKORDER: per-thread lock stacks, global map of observed lock pairs,
// potential_deadlock_detected() reporting both orders, AssertLockHeld/AssertLockNotHeld).
//
// Design: the check is compiled in always and switched on at run time
// (-debuglockorder, or SetLockOrderChecking(true) in tests); when off, lock()/unlock()
// cost one relaxed atomic load.
#pragma once
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

class CCriticalSection : public std::recursive_mutex {
public:
    explicit CCriticalSection(const char* name = "cs") : name(name) {}
    void lock() {
        if (detail::g_lockorder.load(std::memory_order_relaxed)) detail::EnterCritical(this, name);
        std::recursive_mutex::lock();
    }
    void unlock() {
        std::recursive_mutex::unlock();
        if (detail::g_lockorder.load(std::memory_order_relaxed)) detail::LeaveCritical(this);
    }
    bool try_lock() {
        if (!std::recursive_mutex::try_lock()) return false;
        if (detail::g_lockorder.load(std::memory_order_relaxed)) detail::EnterCritical(this, name);
        return true;
    }
    const char* Name() const { return name; }

private:
    const char* name;
};

// Only meaningful while lock-order checking is on.
void AssertLockHeldImpl(const CCriticalSection& cs, const char* file, int line);
void AssertLockNotHeldImpl(const CCriticalSection& cs, const char* file, int line);
#define AssertLockHeld(cs) ::bcp::AssertLockHeldImpl(cs, __FILE__, __LINE__)
#define AssertLockNotHeld(cs) ::bcp::AssertLockNotHeldImpl(cs, __FILE__, __LINE__)

} // namespace bcp
