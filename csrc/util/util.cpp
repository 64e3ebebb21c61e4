#include "util/util.h"
#include "util/strencodings.h"

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <pthread.h>
#include <thread>
#include <sys/stat.h>
#include <unistd.h>

namespace bcp {

// ---------------------------------------------------------------- time
static std::atomic<int64_t> nMockTime{0};

int64_t GetTime() {
    const int64_t m = nMockTime.load();
    if (m) return m;
    return (int64_t)std::chrono::duration_cast<std::chrono::seconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}
int64_t GetTimeMillis() {
    return (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}
int64_t GetTimeMicros() {
    return (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}
int64_t GetSystemTimeInSeconds() { return GetTimeMicros() / 1000000; }
void SetMockTime(int64_t t) { nMockTime = t; }
int64_t GetMockTime() { return nMockTime.load(); }
void MilliSleep(int64_t n) { std::this_thread::sleep_for(std::chrono::milliseconds(n)); }

static std::mutex cs_nTimeOffset;
static int64_t nTimeOffset = 0;
int64_t GetTimeOffset() {
    std::lock_guard<std::mutex> l(cs_nTimeOffset);
    return nTimeOffset;
}
int64_t GetAdjustedTime() { return GetTime() + GetTimeOffset(); }

// Median of peer clock offsets, recomputed at odd sample counts (reference timedata.cpp:44-110;
// at 200 samples the count stays even, so the offset freezes, as there).
bool AddTimeData(const std::string& peer, int64_t nOffsetSample) {
    static std::set<std::string> setKnown;
    static MedianFilter<int64_t> offsets(200, 0);
    static bool fWarned = false;
    std::lock_guard<std::mutex> l(cs_nTimeOffset);
    if (setKnown.size() == 200 || !setKnown.insert(peer).second) return false;
    offsets.input(nOffsetSample);
    LogPrint(BCLog::NET, "added time data, samples %d, offset %+lld (%+lld minutes)\n", offsets.size(),
             (long long)nOffsetSample, (long long)nOffsetSample / 60);
    if (offsets.size() < 5 || offsets.size() % 2 == 0) return false;
    const int64_t median = offsets.median();
    if (std::abs(median) <= std::max<int64_t>(0, gArgs.GetArg("-maxtimeadjustment", DEFAULT_MAX_TIME_ADJUSTMENT))) {
        nTimeOffset = median;
        return false;
    }
    nTimeOffset = 0;
    if (fWarned) return false;
    for (int64_t o : offsets.sorted())
        if (o != 0 && std::abs(o) < 5 * 60) return false; // someone agrees with us
    fWarned = true;
    return true;
}

// ---------------------------------------------------------------- logging
namespace {
struct LogState {
    std::mutex m;
    FILE* file = nullptr;
    std::string path;
    bool console = false;
    bool timestamps = true;
    bool micros = false;
    bool startedNewLine = true;
    std::atomic<uint32_t> categories{0};
};
LogState& L() {
    static LogState s;
    return s;
}
const std::pair<uint32_t, const char*> kCats[] = {
    {BCLog::NET, "net"}, {BCLog::TOR, "tor"}, {BCLog::MEMPOOL, "mempool"}, {BCLog::HTTP, "http"},
    {BCLog::BENCH, "bench"}, {BCLog::ZMQ, "zmq"}, {BCLog::DB, "db"}, {BCLog::RPC, "rpc"},
    {BCLog::ESTIMATEFEE, "estimatefee"}, {BCLog::ADDRMAN, "addrman"}, {BCLog::SELECTCOINS, "selectcoins"},
    {BCLog::REINDEX, "reindex"}, {BCLog::CMPCTBLOCK, "cmpctblock"}, {BCLog::RAND, "rand"}, {BCLog::PRUNE, "prune"},
    {BCLog::PROXY, "proxy"}, {BCLog::MEMPOOLREJ, "mempoolrej"}, {BCLog::LIBEVENT, "libevent"},
    {BCLog::COINDB, "coindb"}, {BCLog::QT, "qt"}, {BCLog::LEVELDB, "leveldb"}, {BCLog::GPU, "gpu"},
    {BCLog::MINING, "mining"}, {BCLog::VALIDATION, "validation"},
};
bool CatFromName(const std::string& n, uint32_t& out) {
    if (n.empty() || n == "1" || n == "all") {
        out = BCLog::ALL;
        return true;
    }
    for (const auto& c : kCats)
        if (n == c.second) {
            out = c.first;
            return true;
        }
    return false;
}
std::string VFormat(const char* fmt, va_list ap) {
    va_list ap2;
    va_copy(ap2, ap);
    const int n = vsnprintf(nullptr, 0, fmt, ap2);
    va_end(ap2);
    std::string s(n > 0 ? (size_t)n : 0, '\0');
    if (n > 0) vsnprintf(&s[0], (size_t)n + 1, fmt, ap);
    return s;
}
} // namespace

bool fLogIPs = false;
void LogSetTimeMicros(bool on) { L().micros = on; }
void LogInit(const std::string& path, bool console, bool timestamps) {
    LogState& s = L();
    std::lock_guard<std::mutex> l(s.m);
    if (s.file) fclose(s.file);
    s.file = path.empty() ? nullptr : fopen(path.c_str(), "a");
    if (s.file) setvbuf(s.file, nullptr, _IOLBF, 0);
    s.path = path;
    s.console = console;
    s.timestamps = timestamps;
}
void LogShutdown() {
    LogState& s = L();
    std::lock_guard<std::mutex> l(s.m);
    if (s.file) fclose(s.file);
    s.file = nullptr;
}
bool LogEnableCategory(const std::string& n) {
    uint32_t f;
    if (!CatFromName(n, f)) return false;
    L().categories |= f;
    return true;
}
bool LogDisableCategory(const std::string& n) {
    uint32_t f;
    if (!CatFromName(n, f)) return false;
    L().categories &= ~f;
    return true;
}
bool LogAcceptCategory(uint32_t c) { return (L().categories.load() & c) != 0; }
uint32_t LogCategories() { return L().categories.load(); }
std::string LogCategoriesString() {
    std::string r;
    for (const auto& c : kCats) r += std::string(r.empty() ? "" : ", ") + c.second;
    return r;
}

void LogPrintStr(const std::string& str) {
    LogState& s = L();
    std::lock_guard<std::mutex> l(s.m);
    std::string out;
    if (s.timestamps && s.startedNewLine) {
        const int64_t us = GetTimeMicros();
        time_t t = (time_t)(us / 1000000);
        struct tm tmv;
        gmtime_r(&t, &tmv);
        char buf[64];
        strftime(buf, sizeof(buf), "%Y-%m-%d %H:%M:%S", &tmv);
        out = s.micros ? strprintf("%s.%06d ", buf, (int)(us % 1000000)) : std::string(buf) + " ";
    }
    out += str;
    s.startedNewLine = !str.empty() && str.back() == '\n';
    if (s.console) {
        fwrite(out.data(), 1, out.size(), stdout);
        fflush(stdout);
    }
    if (s.file) fwrite(out.data(), 1, out.size(), s.file);
}
void LogPrintf(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::string s = VFormat(fmt, ap);
    va_end(ap);
    LogPrintStr(s);
}
void LogPrintCat(uint32_t, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::string s = VFormat(fmt, ap);
    va_end(ap);
    LogPrintStr(s);
}
bool error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::string s = VFormat(fmt, ap);
    va_end(ap);
    LogPrintStr("ERROR: " + s + "\n");
    return false;
}
void ShrinkDebugFile() {
    // keep the last 10 MB of a debug.log larger than 11 MB (reference util.cpp ShrinkDebugFile)
    LogState& s = L();
    std::lock_guard<std::mutex> l(s.m);
    if (s.path.empty()) return;
    const int64_t sz = FileSize(s.path);
    if (sz <= 11 * 1000000) return;
    FILE* f = fopen(s.path.c_str(), "r");
    if (!f) return;
    std::vector<char> buf(10 * 1000000);
    fseek(f, -(long)buf.size(), SEEK_END);
    const size_t n = fread(buf.data(), 1, buf.size(), f);
    fclose(f);
    if (s.file) fclose(s.file);
    f = fopen(s.path.c_str(), "w");
    if (f) {
        fwrite(buf.data(), 1, n, f);
        fclose(f);
    }
    s.file = fopen(s.path.c_str(), "a");
}

// ---------------------------------------------------------------- args
ArgsManager gArgs;

static bool InterpretBool(const std::string& v) { return v.empty() ? true : atoi64(v) != 0; }

void ArgsManager::ParseParameters(int argc, const char* const argv[]) {
    std::lock_guard<CCriticalSection> l(cs_args);
    mapArgs.clear();
    mapMultiArgs.clear();
    for (int i = 1; i < argc; i++) {
        std::string key(argv[i]), value;
        const size_t eq = key.find('=');
        if (eq != std::string::npos) {
            value = key.substr(eq + 1);
            key = key.substr(0, eq);
        }
        if (key.empty() || key[0] != '-') break;
        if (key.size() > 1 && key[1] == '-') key = key.substr(1); // --foo == -foo
        // -nofoo => -foo=0, -nofoo=0 => -foo=1 (reference util.cpp InterpretNegativeSetting)
        if (key.compare(0, 3, "-no") == 0 && key.size() > 3) {
            key = "-" + key.substr(3);
            value = InterpretBool(value) ? "0" : "1";
        }
        mapArgs[key] = value;
        mapMultiArgs[key].push_back(value);
    }
}

bool ArgsManager::ReadConfigFile(const std::string& path) {
    std::ifstream f(path);
    if (!f.good()) return false;
    std::lock_guard<CCriticalSection> l(cs_args);
    std::string line;
    while (std::getline(f, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = TrimString(line);
        if (line.empty()) continue;
        const size_t eq = line.find('=');
        std::string k = TrimString(line.substr(0, eq)), v = eq == std::string::npos ? "1" : TrimString(line.substr(eq + 1));
        const std::string key = "-" + k;
        // command line wins over config
        if (!mapArgs.count(key)) mapArgs[key] = v;
        mapMultiArgs[key].push_back(v);
    }
    return true;
}

std::vector<std::string> ArgsManager::GetArgs(const std::string& a) const {
    std::lock_guard<CCriticalSection> l(cs_args);
    auto it = mapMultiArgs.find(a);
    return it == mapMultiArgs.end() ? std::vector<std::string>() : it->second;
}
bool ArgsManager::IsArgSet(const std::string& a) const {
    std::lock_guard<CCriticalSection> l(cs_args);
    return mapArgs.count(a) > 0;
}
std::string ArgsManager::GetArg(const std::string& a, const std::string& d) const {
    std::lock_guard<CCriticalSection> l(cs_args);
    auto it = mapArgs.find(a);
    return it == mapArgs.end() ? d : it->second;
}
int64_t ArgsManager::GetArg(const std::string& a, int64_t d) const {
    std::lock_guard<CCriticalSection> l(cs_args);
    auto it = mapArgs.find(a);
    return it == mapArgs.end() ? d : atoi64(it->second);
}
bool ArgsManager::GetBoolArg(const std::string& a, bool d) const {
    std::lock_guard<CCriticalSection> l(cs_args);
    auto it = mapArgs.find(a);
    return it == mapArgs.end() ? d : InterpretBool(it->second);
}
bool ArgsManager::SoftSetArg(const std::string& a, const std::string& v) {
    std::lock_guard<CCriticalSection> l(cs_args);
    if (mapArgs.count(a)) return false;
    ForceSetArg(a, v);
    return true;
}
bool ArgsManager::SoftSetBoolArg(const std::string& a, bool v) { return SoftSetArg(a, v ? "1" : "0"); }
void ArgsManager::ForceSetArg(const std::string& a, const std::string& v) {
    std::lock_guard<CCriticalSection> l(cs_args);
    mapArgs[a] = v;
    mapMultiArgs[a] = {v};
}
void ArgsManager::ForceSetMultiArg(const std::string& a, const std::string& v) {
    std::lock_guard<CCriticalSection> l(cs_args);
    mapMultiArgs[a].push_back(v);
}
void ArgsManager::ClearArg(const std::string& a) {
    std::lock_guard<CCriticalSection> l(cs_args);
    mapArgs.erase(a);
    mapMultiArgs.erase(a);
}
std::string ArgsManager::GetChainName() const {
    const bool reg = GetBoolArg("-regtest", false), test = GetBoolArg("-testnet", false);
    if (reg && test) throw std::runtime_error("Invalid combination of -regtest and -testnet.");
    return reg ? "regtest" : test ? "test" : "main";
}

// ---------------------------------------------------------------- filesystem
static std::mutex csDataDir;
static std::string g_dataDir, g_dataDirNet;

std::string GetDefaultDataDir() {
    const char* home = getenv("HOME");
    return std::string(home && *home ? home : "/") + "/.bitcoincashplus";
}
bool TryCreateDirectories(const std::string& p) {
    std::string cur;
    for (size_t i = 0; i < p.size(); i++) {
        cur.push_back(p[i]);
        if ((p[i] == '/' || i + 1 == p.size()) && !cur.empty()) ::mkdir(cur.c_str(), 0700);
    }
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}
void SetDataDir(const std::string& dir) {
    std::lock_guard<std::mutex> l(csDataDir);
    g_dataDir = dir;
    g_dataDirNet.clear();
}
void ClearDatadirCache() {
    std::lock_guard<std::mutex> l(csDataDir);
    g_dataDirNet.clear();
}
std::string GetDataDir(bool fNetSpecific) {
    std::lock_guard<std::mutex> l(csDataDir);
    if (g_dataDir.empty()) g_dataDir = gArgs.GetArg("-datadir", GetDefaultDataDir());
    if (!fNetSpecific) return g_dataDir;
    if (g_dataDirNet.empty()) {
        const std::string chain = gArgs.GetChainName();
        g_dataDirNet = g_dataDir + (chain == "main" ? "" : chain == "test" ? "/testnet3" : "/regtest");
        TryCreateDirectories(g_dataDirNet);
    }
    return g_dataDirNet;
}
bool FileExists(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
}
int64_t FileSize(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0 ? (int64_t)st.st_size : -1;
}
bool RemoveFile(const std::string& p) { return ::unlink(p.c_str()) == 0; }
bool RenameOver(const std::string& src, const std::string& dst) { return ::rename(src.c_str(), dst.c_str()) == 0; }
bool FileCommit(FILE* file) {
    if (fflush(file) != 0) return false;
    return fsync(fileno(file)) == 0;
}
void RenameThread(const char* name) { pthread_setname_np(pthread_self(), std::string(name).substr(0, 15).c_str()); }
int GetNumCores() { return std::max(1u, std::thread::hardware_concurrency()); }
std::string FormatFullVersion() { return "v0.17.0-mi355x"; }
std::string FormatSubVersion(const std::string& name, int nClientVersion, const std::vector<std::string>& comments) {
    std::string s = "/" + name + ":" + strprintf("%d.%d.%d", nClientVersion / 1000000, (nClientVersion / 10000) % 100,
                                                   (nClientVersion / 100) % 100);
    if (!comments.empty()) {
        s += "(";
        for (size_t i = 0; i < comments.size(); i++) s += (i ? "; " : "") + comments[i];
        s += ")";
    }
    return s + "/";
}

// ---------------------------------------------------------------- WorkerPool
WorkerPool::WorkerPool(int nThreads) {
    for (int i = 0; i < nThreads - 1; i++) threads.emplace_back([this] { Loop(); });
}
WorkerPool::~WorkerPool() {
    {
        std::lock_guard<std::mutex> l(m);
        stop = true;
    }
    cv.notify_all();
    for (auto& t : threads) t.join();
}
void WorkerPool::Loop() {
    RenameThread("bcp-worker");
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(m);
    while (true) {
        cv.wait(l, [&] { return stop || (cur != nullptr && generation != seen); });
        if (stop) return;
        seen = generation;
        Job* j = cur;
        j->active++;
        l.unlock();
        while (true) {
            const size_t start = j->next.fetch_add(j->grain);
            if (start >= j->n) break;
            const size_t end = std::min(j->n, start + j->grain);
            for (size_t i = start; i < end; i++) (*j->fn)(i);
        }
        l.lock();
        if (--j->active == 0) cvDone.notify_all();
    }
}
void WorkerPool::ParallelFor(size_t n, const std::function<void(size_t)>& fn, size_t grain) {
    if (n == 0) return;
    if (threads.empty() || n <= grain) {
        for (size_t i = 0; i < n; i++) fn(i);
        return;
    }
    // one call at a time per pool (a nested ParallelFor on the same pool from inside fn would
    // deadlock; fn may use another pool)
    std::lock_guard<std::mutex> one(serialize);
    Job job;
    job.fn = &fn;
    job.n = n;
    job.grain = std::max<size_t>(1, grain);
    {
        std::lock_guard<std::mutex> l(m);
        cur = &job;
        generation++;
    }
    cv.notify_all();
    while (true) {
        const size_t start = job.next.fetch_add(job.grain);
        if (start >= n) break;
        const size_t end = std::min(n, start + job.grain);
        for (size_t i = start; i < end; i++) fn(i);
    }
    // every index is claimed; wait for the workers still inside, then close the call so a
    // worker waking late does not join it
    std::unique_lock<std::mutex> l(m);
    cvDone.wait(l, [&] { return job.active == 0; });
    cur = nullptr;
}

// ---------------------------------------------------------------- Scheduler
Scheduler::Scheduler() : th([this] { Loop(); }) {}
Scheduler::~Scheduler() { Stop(); }
void Scheduler::Stop() {
    {
        std::lock_guard<std::mutex> l(m);
        if (stop) return;
        stop = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
}
void Scheduler::ScheduleEvery(std::function<void()> f, int64_t d) {
    std::lock_guard<std::mutex> l(m);
    tasks.emplace(GetTimeMillis() + d, std::make_pair(std::move(f), d));
    cv.notify_all();
}
void Scheduler::ScheduleFromNow(std::function<void()> f, int64_t d) {
    std::lock_guard<std::mutex> l(m);
    tasks.emplace(GetTimeMillis() + d, std::make_pair(std::move(f), (int64_t)0));
    cv.notify_all();
}
void Scheduler::Loop() {
    RenameThread("bcp-scheduler");
    std::unique_lock<std::mutex> l(m);
    while (!stop) {
        if (tasks.empty()) {
            cv.wait(l);
            continue;
        }
        const int64_t now = GetTimeMillis();
        auto it = tasks.begin();
        if (it->first > now) {
            cv.wait_for(l, std::chrono::milliseconds(it->first - now));
            continue;
        }
        auto task = it->second;
        tasks.erase(it);
        l.unlock();
        try {
            task.first();
        } catch (const std::exception& e) {
            LogPrintf("scheduler task threw: %s\n", e.what());
        }
        l.lock();
        if (task.second > 0) tasks.emplace(GetTimeMillis() + task.second, task);
    }
}

} // namespace bcp

namespace bcp {
void ReplaceAll(std::string& s, const std::string& from, const std::string& to) {
    if (from.empty()) return;
    size_t p = 0;
    while ((p = s.find(from, p)) != std::string::npos) {
        s.replace(p, from.size(), to);
        p += to.size();
    }
}

void RunCommand(const std::string& cmd) {
    const int r = std::system(cmd.c_str());
    if (r != 0) LogPrintf("runCommand error: system(%s) returned %d\n", cmd.c_str(), r);
}

void RunCommandAsync(const std::string& cmd) { std::thread([cmd] { RunCommand(cmd); }).detach(); }
} // namespace bcp

namespace bcp {
static std::atomic<bool> g_gpuFaultInjection{false};
void SetGpuFaultInjection(bool on) { g_gpuFaultInjection = on; }
bool GpuFaultInjection() { return g_gpuFaultInjection.load(); }
} // namespace bcp
