// ThreadSanitizer builds only (Makefile TSAN_FLAGS force-include this header).
// GCC 11's libtsan does not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_for / wait_until on the steady clock. TSan then never sees the mutex
// released and re-acquired inside a timed wait and reports a "double lock" plus data races on
// everything that mutex protects. Without this macro libstdc++ routes those waits through
// pthread_cond_timedwait, which TSan intercepts.
#pragma once
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
