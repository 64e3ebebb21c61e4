// Node runtime utilities: logging with categories, mock/adjusted time, argument/config
// parsing, a fixed worker pool, and thread naming.
// Parity: reference src/util.{h,cpp} (LogPrintf/LogPrint categories, -debug, debug.log,
// mapArgs/mapMultiArgs, ReadConfigFile, GetDataDir), src/utiltime.{h,cpp} (GetTime,
// GetTimeMillis/Micros, SetMockTime), src/timedata.{h,cpp} (GetAdjustedTime, AddTimeData:
// median of up to 200 peer offsets, +-70 minute cap), src/checkqueue.h (worker pool,
// replaced here by ParallelFor), src/scheduler.{h,cpp}.
#pragma once
#include "util/sync.h"
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace bcp {

// ---------------------------------------------------------------- time
int64_t GetTime();        // seconds, mockable
int64_t GetTimeMillis();  // wall clock, not mockable
int64_t GetTimeMicros();
int64_t GetSystemTimeInSeconds();
void SetMockTime(int64_t nMockTimeIn);
int64_t GetMockTime();
void MilliSleep(int64_t n);

int64_t GetTimeOffset();
int64_t GetAdjustedTime();
// Returns true once, the first time the samples disagree with our clock by more than
// -maxtimeadjustment and no peer is within 5 minutes of it (the caller raises the "check your
// computer's date and time" warning, reference timedata.cpp:86-105).
bool AddTimeData(const std::string& peer, int64_t nOffsetSample);
static const char* const CLOCK_WARNING =
    "Please check that your computer's date and time are correct! If your clock is wrong, Bitcoin Cash Plus will "
    "not work properly.";

// Median of the last N values (reference timedata.h CMedianFilter). The window keeps arrival
// order for eviction and a sorted copy updated by one binary-search insert/erase per value.
template <typename T> class MedianFilter {
public:
    MedianFilter(unsigned size, T initial) : nSize(size) {
        window.push_back(initial);
        ordered.push_back(initial);
    }
    void input(T v) {
        if (window.size() == nSize) {
            ordered.erase(std::lower_bound(ordered.begin(), ordered.end(), window.front()));
            window.erase(window.begin());
        }
        window.push_back(v);
        ordered.insert(std::upper_bound(ordered.begin(), ordered.end(), v), v);
    }
    T median() const {
        const size_t n = ordered.size();
        return (n & 1) ? ordered[n / 2] : (ordered[n / 2 - 1] + ordered[n / 2]) / 2;
    }
    int size() const { return (int)window.size(); }
    const std::vector<T>& sorted() const { return ordered; }

private:
    unsigned nSize;
    std::vector<T> window, ordered;
};
static const int64_t DEFAULT_MAX_TIME_ADJUSTMENT = 70 * 60;

// ---------------------------------------------------------------- logging
namespace BCLog {
enum LogFlags : uint32_t {
    NONE = 0, NET = 1 << 0, TOR = 1 << 1, MEMPOOL = 1 << 2, HTTP = 1 << 3, BENCH = 1 << 4, ZMQ = 1 << 5,
    DB = 1 << 6, RPC = 1 << 7, ESTIMATEFEE = 1 << 8, ADDRMAN = 1 << 9, SELECTCOINS = 1 << 10, REINDEX = 1 << 11,
    CMPCTBLOCK = 1 << 12, RAND = 1 << 13, PRUNE = 1 << 14, PROXY = 1 << 15, MEMPOOLREJ = 1 << 16,
    LIBEVENT = 1 << 17, COINDB = 1 << 18, QT = 1 << 19, LEVELDB = 1 << 20, GPU = 1 << 21, MINING = 1 << 22,
    VALIDATION = 1 << 23, ALL = ~(uint32_t)0,
};
}
void LogInit(const std::string& debugLogPath, bool printToConsole, bool logTimestamps = true);
void LogSetTimeMicros(bool on); // -logtimemicros: microsecond timestamps
extern bool fLogIPs;            // -logips: include peer IP addresses in debug output
void LogShutdown();
bool LogEnableCategory(const std::string& name); // "net", "1"/"all"
bool LogDisableCategory(const std::string& name);
bool LogAcceptCategory(uint32_t category);
uint32_t LogCategories();
std::string LogCategoriesString();
void LogPrintStr(const std::string& s);
void LogPrintf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void LogPrintCat(uint32_t cat, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#define LogPrint(cat, ...)                                      \
    do {                                                        \
        if (::bcp::LogAcceptCategory(cat)) ::bcp::LogPrintCat(cat, __VA_ARGS__); \
    } while (0)
bool error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void ShrinkDebugFile();
// Replace every occurrence of `from` in `s` (boost::replace_all in the reference).
void ReplaceAll(std::string& s, const std::string& from, const std::string& to);
// Run a shell command (reference util.cpp runCommand); the async form runs it on a
// detached thread so notification hooks never block validation.
void RunCommand(const std::string& cmd);
void RunCommandAsync(const std::string& cmd);

// ---------------------------------------------------------------- args / config
class ArgsManager {
public:
    void ParseParameters(int argc, const char* const argv[]);
    bool ReadConfigFile(const std::string& path); // key=value lines, '#' comments
    std::vector<std::string> GetArgs(const std::string& strArg) const;
    bool IsArgSet(const std::string& strArg) const;
    std::string GetArg(const std::string& strArg, const std::string& strDefault) const;
    int64_t GetArg(const std::string& strArg, int64_t nDefault) const;
    bool GetBoolArg(const std::string& strArg, bool fDefault) const;
    bool SoftSetArg(const std::string& strArg, const std::string& strValue);
    bool SoftSetBoolArg(const std::string& strArg, bool fValue);
    void ForceSetArg(const std::string& strArg, const std::string& strValue);
    void ForceSetMultiArg(const std::string& strArg, const std::string& strValue);
    void ClearArg(const std::string& strArg);
    std::string GetChainName() const; // main/test/regtest from -testnet/-regtest
    const std::map<std::string, std::string>& Args() const { return mapArgs; }

private:
    mutable CCriticalSection cs_args;
    std::map<std::string, std::string> mapArgs;
    std::map<std::string, std::vector<std::string>> mapMultiArgs;
};
extern ArgsManager gArgs;

std::string GetDefaultDataDir();
std::string GetDataDir(bool fNetSpecific = true);
void SetDataDir(const std::string& dir);
void ClearDatadirCache();
bool TryCreateDirectories(const std::string& p);
bool FileExists(const std::string& p);
int64_t FileSize(const std::string& p);
bool RemoveFile(const std::string& p);
bool RenameOver(const std::string& src, const std::string& dst);
bool FileCommit(FILE* file);
void RenameThread(const char* name);
int GetNumCores();
// -gpufaultinjection (tests only): every GPU batch issued by validation throws, as a failed
// hipMalloc or launch would, so the CPU fallback paths can be exercised on any host.
void SetGpuFaultInjection(bool on);
bool GpuFaultInjection();
std::string FormatFullVersion();
std::string FormatSubVersion(const std::string& name, int nClientVersion, const std::vector<std::string>& comments);
static const int CLIENT_VERSION = 170000; // 0.17.0
static const char* const CLIENT_NAME = "Bitcoin Cash Plus";

// ---------------------------------------------------------------- parallelism
// Fixed pool of worker threads executing index-range jobs; the caller participates.
class WorkerPool {
public:
    explicit WorkerPool(int nThreads);
    ~WorkerPool();
    int Size() const { return (int)threads.size() + 1; }
    // Calls fn(i) for i in [0, n) across the pool; returns when all are done.
    void ParallelFor(size_t n, const std::function<void(size_t)>& fn, size_t grain = 1);

private:
    // One ParallelFor call: lives on the caller's stack until every worker that joined it
    // (active) has left, so a worker never touches a finished call's state.
    struct Job {
        const std::function<void(size_t)>* fn;
        size_t n, grain;
        std::atomic<size_t> next{0};
        int active = 0; // workers inside this job (guarded by m)
    };
    void Loop();
    std::vector<std::thread> threads;
    std::mutex m, serialize;
    std::condition_variable cv, cvDone;
    Job* cur = nullptr; // the open call, if any (guarded by m)
    uint64_t generation = 0;
    bool stop = false;
};

// Periodic / delayed task thread (reference CScheduler).
class Scheduler {
public:
    Scheduler();
    ~Scheduler();
    void ScheduleEvery(std::function<void()> f, int64_t deltaMillis);
    void ScheduleFromNow(std::function<void()> f, int64_t deltaMillis);
    void Stop();

private:
    void Loop();
    std::multimap<int64_t, std::pair<std::function<void()>, int64_t>> tasks; // due -> (fn, period)
    std::mutex m;
    std::condition_variable cv;
    bool stop = false;
    std::thread th;
};

// Interruptible sleep shared by background threads (reference CThreadInterrupt).
class ThreadInterrupt {
public:
    explicit operator bool() const { return flag.load(); }
    void operator()() {
        {
            std::lock_guard<std::mutex> l(m);
            flag = true;
        }
        cv.notify_all();
    }
    void reset() { flag = false; }
    bool sleep_for(int64_t millis) {
        std::unique_lock<std::mutex> l(m);
        return !cv.wait_for(l, std::chrono::milliseconds(millis), [this] { return flag.load(); });
    }

private:
    std::condition_variable cv;
    std::mutex m;
    std::atomic<bool> flag{false};
};

} // namespace bcp
