// Clang thread-safety annotations (reference src/threadsafety.h:16-60). Under clang with
// -Wthread-safety (`make thread-safety`) the analysis checks at compile time that guarded members
// are only touched with their mutex held and that functions documented as needing a lock are
// only called with it; under GCC every macro expands to nothing.
#pragma once

#if defined(__clang__)
#define BCP_TSA(x) __attribute__((x))
#else
#define BCP_TSA(x)
#endif

#define CAPABILITY(x) BCP_TSA(capability(x))
#define SCOPED_CAPABILITY BCP_TSA(scoped_lockable)
#define GUARDED_BY(x) BCP_TSA(guarded_by(x))
#define PT_GUARDED_BY(x) BCP_TSA(pt_guarded_by(x))
#define ACQUIRED_BEFORE(...) BCP_TSA(acquired_before(__VA_ARGS__))
#define ACQUIRED_AFTER(...) BCP_TSA(acquired_after(__VA_ARGS__))
#define EXCLUSIVE_LOCKS_REQUIRED(...) BCP_TSA(exclusive_locks_required(__VA_ARGS__))
#define SHARED_LOCKS_REQUIRED(...) BCP_TSA(shared_locks_required(__VA_ARGS__))
#define LOCKS_EXCLUDED(...) BCP_TSA(locks_excluded(__VA_ARGS__))
#define ACQUIRE(...) BCP_TSA(acquire_capability(__VA_ARGS__))
#define RELEASE(...) BCP_TSA(release_capability(__VA_ARGS__))
#define TRY_ACQUIRE(...) BCP_TSA(try_acquire_capability(__VA_ARGS__))
#define ASSERT_EXCLUSIVE_LOCK(...) BCP_TSA(assert_exclusive_lock(__VA_ARGS__))
#define RETURN_CAPABILITY(x) BCP_TSA(lock_returned(x))
#define NO_THREAD_SAFETY_ANALYSIS BCP_TSA(no_thread_safety_analysis)
