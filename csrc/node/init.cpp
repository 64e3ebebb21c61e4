#include "node/init.h"

#include <thread>
#include "node/ui_interface.h"
#include "consensus/params.h"
#include "consensus/versionbits.h"
#include "kernels/gpu_api.h"
#include "node/gpuverify.h"
#include "node/miner.h"
#include "node/node.h"
#include "node/policy.h"
#include "node/sigverify.h"
#include "net/blockencodings.h"
#include "rpc/httpserver.h"
#include "rpc/server.h"
#include "script/standard.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <csignal>
#include <execinfo.h>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

namespace bcp {

// Subsystem hooks: strong definitions live in the net / wallet / zmq modules.
__attribute__((weak)) bool StartNetwork(NodeContext&, std::string&) { return true; }
__attribute__((weak)) void StopNetwork(NodeContext&) {}
__attribute__((weak)) bool StartWallet(NodeContext&, std::string&) { return true; }
__attribute__((weak)) void StopWallet(NodeContext&) {}
__attribute__((weak)) bool StartZMQ(NodeContext&, std::string&) { return true; }
__attribute__((weak)) void StopZMQ(NodeContext&) {}
__attribute__((weak)) std::string NetHelp() { return ""; }
__attribute__((weak)) std::string WalletHelp() { return ""; }

std::string HelpMessage() {
    std::string s = "Usage:\n  bcpd [options]                     Start Bitcoin Cash Plus Daemon (MI355X build)\n\nOptions:\n";
    const std::pair<const char*, const char*> opts[] = {
        {"-?", "Print this help message and exit"},
        {"-version", "Print version and exit"},
        {"-conf=<file>", "Specify configuration file (default: bitcoincashplus.conf)"},
        {"-datadir=<dir>", "Specify data directory"},
        {"-daemon", "Run in the background as a daemon and accept commands"},
        {"-pid=<file>", "Specify pid file (default: bitcoincashplusd.pid)"},
        {"-testnet", "Use the test chain"},
        {"-regtest", "Enter regression test mode (Equihash 48,5; fork at height 3000)"},
        {"-dbcache=<n>", "Set database cache size in megabytes (default: 450)"},
        {"-par=<n>", "Number of script verification threads (0 = auto)"},
        {"-gpu=<0|1>", "Use the MI355X for batched ECDSA / Equihash verification and mining (default: 1)"},
        {"-gpusigthreshold=<n>", "Minimum signatures per block routed to the GPU verifier (default: 128)"},
        {"-gpushortidthreshold=<n>", "Smallest mempool whose compact-block short ids are computed on the GPU (default: 16384)"},
        {"-gpudevices=<list>", "Comma-separated GPU indices the built-in Equihash miner runs on, one host thread per device (default: all visible)"},
        {"-gpuvalidationdevices=<list>", "Comma-separated GPU indices that verify block signatures and header solutions, one high-priority stream, service thread and host-fill worker group each; batches are sharded across them. When set, the built-in miner leaves these devices alone if others are available (default: every visible device, two lanes each)"},
        {"-maxsigcachesize=<n>", "Limit size of signature cache to <n> MiB (default: 32)"},
        {"-maxscriptcachesize=<n>", "Limit size of script cache to <n> MiB (default: 32)"},
        {"-blocknotify=<cmd>", "Execute command when the best block changes (%s in cmd is replaced by block hash)"},
        {"-bip9params=<deployment>:<start>:<end>", "Use given start/end times for specified version bits deployment (regtest-only)"},
        {"-loadblock=<file>", "Imports blocks from external blk000??.dat file on startup"},
        {"-disablesafemode", "Disable safemode, override a real safe mode event (default: 0)"},
        {"-testsafemode", "Force safe mode (default: 0)"},
        {"-alertnotify=<cmd>", "Execute command when a relevant alert is received or we see a really long fork (%s in cmd is replaced by message)"},
        {"-txindex", "Maintain a full transaction index (default: 0)"},
        {"-prune=<n>", "Reduce storage by pruning old blocks (MiB target, >= 550)"},
        {"-reindex", "Rebuild chain state and block index from the blk*.dat files on disk"},
        {"-reindex-chainstate", "Rebuild chain state from the currently indexed blocks"},
        {"-checkblocks=<n>", "How many blocks to check at startup (default: 6, 0 = all)"},
        {"-checklevel=<n>", "How thorough the block verification of -checkblocks is (0-4, default: 3)"},
        {"-maxmempool=<n>", "Keep the transaction memory pool below <n> megabytes (default: 300)"},
        {"-mempoolexpiry=<n>", "Do not keep transactions in the mempool longer than <n> hours (default: 336)"},
        {"-persistmempool", "Whether to save the mempool on shutdown and load on restart (default: 1)"},
        {"-excessiveblocksize=<n>", "Do not accept blocks larger than this limit, in bytes (default: 8000000)"},
        {"-blockmaxsize=<n>", "Set maximum block size in bytes for mining (default: 2000000)"},
        {"-blockprioritypercentage=<n>", "Set maximum percentage of a block reserved to high-priority transactions (default: 5)"},
        {"-blockmintxfee=<amt>", "Set lowest fee rate (BCP/kB) for transactions to be included in block creation"},
        {"-minrelaytxfee=<amt>", "Fees (BCP/kB) smaller than this are considered zero fee for relaying (default: 0.00001)"},
        {"-dustrelayfee=<amt>", "Fee rate (BCP/kB) used to define dust, the value of an output such that it will cost about 1/3 of its value in fees at this fee rate to spend it (default: 0.00001)"},
        {"-incrementalrelayfee=<amt>", "Fee rate (BCP/kB) used to define cost of relay, used for mempool limiting and BIP 125 replacement (default: 0.00001)"},
        {"-zmqpubhashblock=<address>", "Enable publish hash block in <address>"},
        {"-zmqpubhashtx=<address>", "Enable publish hash transaction in <address>"},
        {"-zmqpubrawblock=<address>", "Enable publish raw block in <address>"},
        {"-zmqpubrawtx=<address>", "Enable publish raw transaction in <address>"},
        {"-datacarrier", "Relay and mine data carrier transactions (default: 1)"},
        {"-datacarriersize=<n>", "Maximum size of data in data carrier transactions (default: 83)"},
        {"-permitbaremultisig", "Relay non-P2SH multisig (default: 1)"},
        {"-usecashaddr", "Use Cash Address for destination encoding instead of base58 (activate by default on Jan, 14) (default: 0)"},
        {"-server", "Accept command line and JSON-RPC commands (default: 1 for bcpd)"},
        {"-rest", "Accept public REST requests (default: 0)"},
        {"-webgui", "Serve the browser wallet GUI at http://<rpcbind>:<rpcport>/gui to authenticated RPC users (default: 0)"},
        {"-rpcbind=<addr>[:port]", "Bind to given address to listen for JSON-RPC connections"},
        {"-rpcport=<port>", "Listen for JSON-RPC connections on <port> (default: 8332 / testnet and regtest 18332)"},
        {"-rpcallowip=<ip>", "Allow JSON-RPC connections from specified source (IP or subnet)"},
        {"-rpcuser=<user>", "Username for JSON-RPC connections"},
        {"-rpcpassword=<pw>", "Password for JSON-RPC connections"},
        {"-rpcauth=<userpw>", "Username and hashed password for JSON-RPC connections (user:salt$hmac)"},
        {"-rpcthreads=<n>", "Set the number of threads to service RPC calls (default: 4)"},
        {"-rpcservertimeout=<n>", "Timeout during HTTP requests (default: 30)"},
        {"-debug=<category>", "Output debugging information (net, mempool, http, bench, rpc, gpu, ...)"},
        {"-printtoconsole", "Send trace/debug info to console instead of debug.log file"},
        {"-logtimestamps", "Prepend debug output with timestamp (default: 1)"},
        {"-logtimemicros", "Add microsecond precision to debug timestamps (default: 0)"},
        {"-logips", "Include IP addresses in debug output (default: 0)"},
        {"-shrinkdebugfile", "Shrink debug.log file on client startup (default: 1)"},
        {"-fastprune", "Use 64 KiB block files (regtest only; for pruning tests)"},
        {"-blockcachemb=<n>", "Keep blocks accepted out of order in memory until they connect, up to <n> MiB "
                              "(decoded in-memory size, several times the serialized size; default: 512; 0 reads them back "
                              "from disk like the reference)"},
        {"-parallelutxo=<n>", "Run the UTXO pass of blocks with at least <n> transactions on all script threads "
                              "(default: 64; 0 = always serial)"},
        {"-connectinplace", "Let that parallel UTXO pass update the coins tip in place, undone from the block's undo "
                            "data if a later check fails, instead of merging a per-block view into it (default: 1)"},
        {"-connectlookahead", "While a block's signatures are checked on the GPU, fetch the next block's input coins and "
                              "precompute its transactions on the idle script threads (default: 1)"},
        {"-acceptnonstdtxn", "Relay and mine \"non-standard\" transactions (default: 0 on main, 1 on the test chains)"},
        {"-assumevalid=<hex>", "If this block is in the chain assume that it and its ancestors are valid and potentially skip their script verification (0 to verify all)"},
        {"-bytespersigop=<n>", "Equivalent bytes per sigop in transactions for relay and mining (default: 20)"},
        {"-checkpoints", "Disable expensive verification for known chain history (default: 1)"},
        {"-debugexclude=<category>", "Exclude debugging information for a category; takes priority over -debug"},
        {"-debuglockorder", "Check lock-order consistency of the node's mutexes (default: 0)"},
        {"-debuglockorderabort", "Abort on a detected lock-order inversion (with -debuglockorder; default: 1)"},
        {"-limitancestorcount=<n>", "Do not accept transactions if the number of in-mempool ancestors is <n> or more (default: 25)"},
        {"-limitancestorsize=<n>", "Do not accept transactions whose size with all in-mempool ancestors exceeds <n> kilobytes (default: 101)"},
        {"-limitdescendantcount=<n>", "Do not accept transactions if any ancestor would have <n> or more in-mempool descendants (default: 25)"},
        {"-limitdescendantsize=<n>", "Do not accept transactions if any ancestor would have more than <n> kilobytes of in-mempool descendants (default: 101)"},
        {"-maxtimeadjustment=<n>", "Maximum allowed median peer time offset adjustment, in seconds (default: 4200)"},
        {"-maxtipage=<n>", "Maximum tip age in seconds to consider the node in initial block download (default: 86400)"},
        {"-maxtxfee=<amt>", "Maximum total fees (in BCP) to use in a single wallet transaction or raw transaction (default: 0.1)"},
        {"-promiscuousmempoolflags=<n>", "Script verification flags for mempool acceptance (testing only)"},
        {"-blockversion=<n>", "Override block version to test forking scenarios (regtest)"},
        {"-sysperms", "Create new files with system default permissions, instead of umask 077 (only effective with disabled wallet functionality)"},
        {"-rpccookiefile=<loc>", "Location of the auth cookie (default: data dir)"},
        {"-rpcworkqueue=<n>", "Set the depth of the work queue to service RPC calls (default: 16)"},
        {"-help-debug", "Show all debugging options (usage: --help -help-debug)"},
        {"-nodebug", "Turn off debugging messages, same as -debug=0"},
    };
    for (const auto& o : opts) s += strprintf("  %-32s %s\n", o.first, o.second);
    // debug-only options, shown with -help-debug (reference init.cpp:306 showDebug)
    if (gArgs.GetBoolArg("-help-debug", false)) {
        const std::pair<const char*, const char*> dbg[] = {
            {"-mocktime=<n>", "Replace actual time with <n> seconds since epoch (default: 0)"},
            {"-stopafterblockimport", "Stop running after importing blocks from disk (default: 0)"},
            {"-printpriority", "Log transaction priority and fee per kB when mining blocks (default: 0)"},
            {"-limitfreerelay=<n>", "Continuously rate-limit free transactions to <n>*1000 bytes per minute (default: 0)"},
            {"-relaypriority", "Require high priority for relaying free or low-fee transactions (default: 1)"},
            {"-checkblockindex", "Do a full consistency check for mapBlockIndex, setBlockIndexCandidates, chainActive and mapBlocksUnlinked occasionally (default: 1 on regtest)"},
            {"-checkmempool=<n>", "Run checks every <n> transactions (default: 1 on regtest)"},
            {"-dropmessagestest=<n>", "Randomly drop 1 of every <n> network messages"},
            {"-fuzzmessagestest=<n>", "Randomly fuzz 1 of every <n> network messages"},
            {"-gpufaultinjection", "Make every validation GPU batch fail so the CPU fallback runs (default: 0)"},
        };
        s += "\nDebugging/Testing options:\n";
        for (const auto& o : dbg) s += strprintf("  %-32s %s\n", o.first, o.second);
    }
    s += NetHelp();
    s += WalletHelp();
    return s;
}

static int g_lockFd = -1;
static bool LockDataDirectory(const std::string& datadir) {
    const std::string path = datadir + "/.lock";
    g_lockFd = open(path.c_str(), O_RDWR | O_CREAT, 0600);
    if (g_lockFd < 0) return false;
    return flock(g_lockFd, LOCK_EX | LOCK_NB) == 0;
}

static std::atomic<bool> g_signalled{false};

// Fatal-signal reporter: symbolised backtrace to stderr (failure diagnostics; the
// reference relies on core dumps).
static void HandleFatalSignal(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char* name = sig == SIGSEGV ? "SIGSEGV" : sig == SIGABRT ? "SIGABRT" : sig == SIGBUS ? "SIGBUS" : "SIGFPE";
    (void)!write(2, "\n*** fatal signal ", 18);
    (void)!write(2, name, strlen(name));
    (void)!write(2, " ***\n", 5);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
static void HandleSIGTERM(int) {
    g_signalled = true;
}

static bool ParseFeeArg(const char* name, CFeeRate& out) {
    if (!gArgs.IsArgSet(name)) return true;
    int64_t n = 0;
    if (!ParseMoney(gArgs.GetArg(name, ""), n)) return false;
    out = CFeeRate(n);
    return true;
}

int AppMain(int argc, char* argv[]) {
    gArgs.ParseParameters(argc, argv);
    if (gArgs.IsArgSet("-?") || gArgs.IsArgSet("-h") || gArgs.IsArgSet("-help")) {
        printf("%s", HelpMessage().c_str());
        return 0;
    }
    if (gArgs.IsArgSet("-version")) {
        printf("%s version %s\n", CLIENT_NAME, FormatFullVersion().c_str());
        return 0;
    }
    const std::string datadirBase = gArgs.GetArg("-datadir", GetDefaultDataDir());
    if (!TryCreateDirectories(datadirBase)) {
        fprintf(stderr, "Error: Specified data directory \"%s\" does not exist.\n", datadirBase.c_str());
        return 1;
    }
    SetDataDir(datadirBase);
    gArgs.ReadConfigFile(datadirBase + "/" + gArgs.GetArg("-conf", "bitcoincashplus.conf"));
    std::string chain;
    try {
        chain = gArgs.GetChainName();
    } catch (const std::exception& e) {
        fprintf(stderr, "Error: %s\n", e.what());
        return 1;
    }
    SelectParams(chain);
    // new files private unless -sysperms (reference init.cpp:1244); the wallet refuses -sysperms
    if (!gArgs.GetBoolArg("-sysperms", false)) umask(077);
    // -bip9params=deployment:start:end, regtest only (reference chainparams.cpp:474
    // UpdateRegtestBIP9Parameters + init.cpp parsing)
    for (const std::string& p : gArgs.GetArgs("-bip9params")) {
        if (chain != "regtest") {
            fprintf(stderr, "Error: BIP9 parameters may only be overridden on regtest.\n");
            return 1;
        }
        const size_t a = p.find(':'), b = a == std::string::npos ? a : p.find(':', a + 1);
        int64_t nStart = 0, nTimeout = 0;
        if (b == std::string::npos || !ParseInt64(p.substr(a + 1, b - a - 1), &nStart) ||
            !ParseInt64(p.substr(b + 1), &nTimeout)) {
            fprintf(stderr, "Error: Version bits parameters malformed, expecting deployment:start:end\n");
            return 1;
        }
        const std::string name = p.substr(0, a);
        bool found = false;
        for (int j = 0; j < (int)Consensus::MAX_VERSION_BITS_DEPLOYMENTS; ++j) {
            if (name == VersionBitsDeploymentInfo[j].name) {
                Params(chain).UpdateVersionBitsParameters((Consensus::DeploymentPos)j, nStart, nTimeout);
                found = true;
                LogPrintf("Setting BIP9 activation parameters for %s to start=%lld, timeout=%lld\n", name.c_str(),
                          (long long)nStart, (long long)nTimeout);
                break;
            }
        }
        if (!found) {
            fprintf(stderr, "Error: Invalid deployment (%s)\n", name.c_str());
            return 1;
        }
    }
    const std::string datadir = GetDataDir(true);
    TryCreateDirectories(datadir);

    // daemonize before any GPU/thread initialisation (fork without exec)
    if (gArgs.GetBoolArg("-daemon", false)) {
        fprintf(stdout, "Bitcoin Cash Plus server starting\n");
        fflush(stdout);
        const pid_t pid = fork();
        if (pid < 0) {
            fprintf(stderr, "Error: fork() returned %d errno %d\n", pid, errno);
            return 1;
        }
        if (pid > 0) return 0;
        setsid();
    }
    // sanity checks (reference AppInitSanityChecks / InitSanityCheck)
    if (!ECC_InitSanityCheck()) {
        InitError("Elliptic curve cryptography sanity check failure. Aborting.");
        return 1;
    }
    if (!Random_SanityCheck()) {
        InitError("OS cryptographic RNG sanity check failure. Aborting.");
        return 1;
    }
    if (!LockDataDirectory(datadir)) {
        fprintf(stderr, "Error: Cannot obtain a lock on data directory %s. Bitcoin Cash Plus is probably already running.\n",
                datadir.c_str());
        return 1;
    }
    const bool console = gArgs.GetBoolArg("-printtoconsole", false);
    if (gArgs.GetBoolArg("-shrinkdebugfile", true) && !console) {
        LogInit(datadir + "/debug.log", false);
        ShrinkDebugFile();
    }
    LogInit(console ? "" : datadir + "/debug.log", console, gArgs.GetBoolArg("-logtimestamps", true));
    LogSetTimeMicros(gArgs.GetBoolArg("-logtimemicros", false));
    fLogIPs = gArgs.GetBoolArg("-logips", false);
    {
        // -debug=0 / -nodebug turn debugging off (reference init.cpp:1327-1334)
        const std::vector<std::string> cats = gArgs.GetArgs("-debug");
        if (!gArgs.GetBoolArg("-nodebug", false) && std::find(cats.begin(), cats.end(), "0") == cats.end())
            for (const std::string& c : cats)
                if (!LogEnableCategory(c)) LogPrintf("Unsupported logging category -debug=%s.\n", c.c_str());
    }
    for (const std::string& c : gArgs.GetArgs("-debugexclude")) LogDisableCategory(c);
    LogPrintf("\n\n\n\n\n");
    LogPrintf("%s version %s (MI355X)\n", CLIENT_NAME, FormatFullVersion().c_str());
    LogPrintf("Using data directory %s\n", datadir.c_str());
    noui_connect();
    uiInterface.InitMessage.connect(SetRPCWarmupStatus);

    {
        const std::string pidfile = datadir + "/" + gArgs.GetArg("-pid", "bitcoincashplusd.pid");
        if (FILE* f = fopen(pidfile.c_str(), "w")) {
            fprintf(f, "%d\n", (int)getpid());
            fclose(f);
        }
    }
    if (gArgs.GetBoolArg("-debuglockorder", false)) SetLockOrderChecking(true, gArgs.GetBoolArg("-debuglockorderabort", true));
    signal(SIGTERM, HandleSIGTERM);
    signal(SIGINT, HandleSIGTERM);
    signal(SIGPIPE, SIG_IGN);
    if (!getenv("BCP_NO_CRASH_HANDLER")) {
        // alternate stack so a stack overflow can still be reported
        static std::vector<char> altstack(1 << 16);
        stack_t ss = {};
        ss.ss_sp = altstack.data();
        ss.ss_size = altstack.size();
        sigaltstack(&ss, nullptr);
        struct sigaction sa = {};
        sa.sa_handler = HandleFatalSignal;
        sa.sa_flags = SA_ONSTACK;
        for (int sig : {SIGSEGV, SIGABRT, SIGBUS, SIGFPE}) sigaction(sig, &sa, nullptr);
    }

    // obsolete options (reference init.cpp:1336-1358)
    if (gArgs.GetBoolArg("-debugnet", false)) InitWarning("Unsupported argument -debugnet ignored, use -debug=net.");
    if (gArgs.IsArgSet("-socks")) {
        InitError("Unsupported argument -socks found. Setting SOCKS version isn't possible anymore, only SOCKS5 proxies are "
                  "supported.");
        return 1;
    }
    if (gArgs.GetBoolArg("-tor", false)) {
        InitError("Unsupported argument -tor found, use -onion.");
        return 1;
    }
    if (gArgs.GetBoolArg("-benchmark", false)) InitWarning("Unsupported argument -benchmark ignored, use -debug=bench.");
    if (gArgs.GetBoolArg("-whitelistalwaysrelay", false))
        InitWarning("Unsupported argument -whitelistalwaysrelay ignored, use -whitelistrelay and/or -whitelistforcerelay.");
    if (gArgs.IsArgSet("-blockminsize")) InitWarning("Unsupported argument -blockminsize ignored.");
    if (gArgs.GetBoolArg("-rpcssl", false)) {
        InitError("SSL mode for RPC (-rpcssl) is no longer supported.");
        return 1;
    }
    // regression tests start with a fixed clock (reference init.cpp:1522)
    SetMockTime(gArgs.GetArg("-mocktime", 0));

    // ---- parameter interaction (policy globals)
    const CChainParams& params = Params();
        fIsBareMultisigStd = gArgs.GetBoolArg("-permitbaremultisig", DEFAULT_PERMIT_BAREMULTISIG);
    fAcceptDatacarrier = gArgs.GetBoolArg("-datacarrier", DEFAULT_ACCEPT_DATACARRIER);
    nMaxDatacarrierBytes = (unsigned)gArgs.GetArg("-datacarriersize", (int64_t)nMaxDatacarrierBytes);
    nBytesPerSigOp = (unsigned)gArgs.GetArg("-bytespersigop", (int64_t)nBytesPerSigOp);
    SetUseCashAddr(gArgs.GetBoolArg("-usecashaddr", false)); // reference src/init.cpp:2119-2120
    if (!ParseFeeArg("-minrelaytxfee", minRelayTxFee) || !ParseFeeArg("-dustrelayfee", dustRelayFee) ||
        !ParseFeeArg("-incrementalrelayfee", incrementalRelayFee)) {
        InitError("Invalid fee amount argument");
        return 1;
    }
    // excessive block size vs the legacy 1MB limit and the mining limit (reference init.cpp
    // AppInitParameterInteraction :1413-1424, config.cpp SetMaxBlockSize)
    {
        const int64_t ebs = gArgs.GetArg("-excessiveblocksize", (int64_t)DEFAULT_MAX_BLOCK_SIZE);
        if (ebs <= (int64_t)LEGACY_MAX_BLOCK_SIZE) {
            InitError("Excessive block size must be > 1,000,000 bytes (1MB)");
            return 1;
        }
        if (gArgs.GetArg("-blockmaxsize", (int64_t)DEFAULT_MAX_GENERATED_BLOCK_SIZE) > ebs) {
            InitError("Max generated block size (blockmaxsize) cannot exceed the excessive block size "
                      "(excessiveblocksize)");
            return 1;
        }
    }
    SetGpuSigThreshold((size_t)gArgs.GetArg("-gpusigthreshold", (int64_t)GetGpuSigThreshold()));
    SetGpuShortIdThreshold((size_t)gArgs.GetArg("-gpushortidthreshold", (int64_t)GetGpuShortIdThreshold()));
    if (gArgs.IsArgSet("-gpudevices")) {
        std::vector<int> devs;
        for (const std::string& tok : SplitString(gArgs.GetArg("-gpudevices", ""), ',')) {
            if (tok.empty()) continue;
            int64_t d = 0;
            if (!ParseInt64(tok, &d) || d < 0) {
                InitError("Invalid -gpudevices entry: " + tok);
                return 1;
            }
            devs.push_back((int)d);
        }
        SetMinerGpuDevices(devs);
    }
    if (gArgs.IsArgSet("-gpuvalidationdevices")) {
        std::vector<int> devs;
        for (const std::string& tok : SplitString(gArgs.GetArg("-gpuvalidationdevices", ""), ',')) {
            if (tok.empty()) continue;
            int64_t d = 0;
            if (!ParseInt64(tok, &d) || d < 0 || d >= 64) {
                InitError("Invalid -gpuvalidationdevices entry: " + tok);
                return 1;
            }
            devs.push_back((int)d);
        }
        GpuVerifyService::Instance().SetDevices(devs);
    }
    InitSignatureCache(gArgs.GetArg("-maxsigcachesize", (int64_t)DEFAULT_MAX_SIG_CACHE_SIZE));
    InitScriptExecutionCache(gArgs.GetArg("-maxscriptcachesize", (int64_t)DEFAULT_MAX_SCRIPT_CACHE_SIZE));
    SetGpuFaultInjection(gArgs.GetBoolArg("-gpufaultinjection", false));
    const bool useGpu = gArgs.GetBoolArg("-gpu", true) && (GpuFaultInjection() || gpu::GpuAvailable());
    LogPrintf("GPU acceleration: %s%s\n", !useGpu ? "disabled" : gpu::GpuAvailable() ? gpu::DeviceName(0).c_str() : "none",
              GpuFaultInjection() ? " (fault injection: every GPU batch fails)" : "");

    // ---- RPC server starts in warmup so clients get RPC_IN_WARMUP while loading
    RegisterAllRPCCommands(tableRPC);
    std::unique_ptr<HTTPServer> http;
    if (gArgs.GetBoolArg("-server", true)) {
        HTTPServer::Options ho;
        const int defaultPort = (int)gArgs.GetArg("-rpcport", (int64_t)params.GetRPCPort());
        std::vector<std::string> binds = gArgs.GetArgs("-rpcbind");
        if (binds.empty() || !gArgs.IsArgSet("-rpcallowip")) {
            ho.bind.push_back({"127.0.0.1", defaultPort});
            ho.bind.push_back({"::1", defaultPort});
        } else {
            for (const std::string& b : binds) {
                const size_t colon = b.rfind(':');
                if (colon != std::string::npos && b.find(':') == colon)
                    ho.bind.push_back({b.substr(0, colon), atoi(b.substr(colon + 1).c_str())});
                else
                    ho.bind.push_back({b, defaultPort});
            }
        }
        ho.allowSubnets = gArgs.GetArgs("-rpcallowip");
        if (!ho.allowSubnets.empty()) {
            ho.allowSubnets.push_back("127.0.0.1");
            ho.allowSubnets.push_back("::1");
        }
        ho.threads = (int)gArgs.GetArg("-rpcthreads", (int64_t)4);
        ho.timeoutSeconds = (int)gArgs.GetArg("-rpcservertimeout", (int64_t)30);
        ho.workQueueDepth = (int)std::max<int64_t>(gArgs.GetArg("-rpcworkqueue", (int64_t)16), 1);
        LogPrintf("HTTP: creating work queue of depth %d\n", ho.workQueueDepth);
        http.reset(new HTTPServer(ho));
        std::string err;
        // handlers first, then the listener (reference AppInitServers: StartHTTPRPC and StartREST
        // before StartHTTPServer), so no early request meets an empty 404
        if (!StartHTTPRPC(*http, datadir, err)) {
            InitError(err);
            return 1;
        }
        if (gArgs.GetBoolArg("-rest", false)) StartREST(*http);
        if (gArgs.GetBoolArg("-webgui", false)) StartWebGUI(*http);
        if (!http->Start(err)) {
            InitError(err);
            return 1;
        }
    }

    // ---- chainstate
    uiInterface.InitMessage("Loading block index...");
    const bool reindex = gArgs.GetBoolArg("-reindex", false) || gArgs.GetBoolArg("-reindex-chainstate", false);
    std::string err;
    std::unique_ptr<NodeContext> node;
    {
        const bool wipe = reindex;
        node = BuildNode(chain, datadir, false, wipe, useGpu);
        SetNode(node.get());
        node->scheduler.reset(new Scheduler());
        if (reindex) {
            uiInterface.InitMessage("Reindexing blocks...");
            if (!node->chainstate->Reindex()) {
                InitError("Reindex failed");
                return 1;
            }
        } else {
            if (!node->chainstate->LoadBlockIndex(err) || !node->chainstate->InitBlockIndex(err)) {
                InitError(err);
                return 1;
            }
        }
        uiInterface.InitMessage("Verifying blocks...");
        if (!node->chainstate->RewindBlockIndex()) LogPrintf("Warning: RewindBlockIndex failed\n");
        if (!node->chainstate->VerifyDB((int)gArgs.GetArg("-checklevel", (int64_t)DEFAULT_CHECKLEVEL),
                                        (int)gArgs.GetArg("-checkblocks", (int64_t)DEFAULT_CHECKBLOCKS))) {
            InitError("Corrupted block database detected. Please restart with -reindex.");
            return 1;
        }
    }
    if (node->mempool && node->mempool->Estimator()) node->mempool->Estimator()->Read(datadir + "/fee_estimates.dat");
    if (gArgs.GetBoolArg("-persistmempool", true)) {
        uiInterface.InitMessage("Loading mempool...");
        node->chainstate->LoadMempool(datadir + "/mempool.dat");
    }
    // Block import (reference init.cpp ThreadImport :974-1046): <datadir>/bootstrap.dat (then
    // renamed to bootstrap.dat.old) and every -loadblock=<file>, on a background thread so RPC
    // and the network come up meanwhile; blocks are accepted, stored and connected as usual.
    std::vector<std::pair<std::string, bool>> importFiles; // (path, is <datadir>/bootstrap.dat)
    {
        const std::string boot = datadir + "/bootstrap.dat";
        FILE* f = fopen(boot.c_str(), "rb");
        if (f) {
            fclose(f);
            importFiles.emplace_back(boot, true);
        }
    }
    for (const std::string& f : gArgs.GetArgs("-loadblock")) importFiles.emplace_back(f, false);
    std::thread importThread;
    if (!importFiles.empty()) {
        importThread = std::thread([files = importFiles, cs = node->chainstate.get()] {
            RenameThread("bcp-loadblk");
            for (const auto& item : files) {
                const std::string& path = item.first;
                FILE* f = fopen(path.c_str(), "rb");
                if (!f) {
                    LogPrintf("Warning: Could not open blocks file %s\n", path.c_str());
                    continue;
                }
                LogPrintf("Importing blocks file %s...\n", path.c_str());
                cs->LoadExternalBlockFile(f); // closes nothing: we own f
                fclose(f);
                if (item.second) {
                    const std::string old = path + ".old";
                    if (rename(path.c_str(), old.c_str()) == 0) LogPrintf("Renamed %s to %s\n", path.c_str(), old.c_str());
                }
            }
            CValidationState state;
            cs->ActivateBestChain(state);
            LogPrintf("Block import finished\n");
            if (gArgs.GetBoolArg("-stopafterblockimport", false)) { // reference init.cpp:1039
                LogPrintf("Stopping after block import\n");
                RequestShutdown();
            }
        });
    }
    uiInterface.InitMessage("Loading wallet...");
    if (!StartWallet(*node, err)) {
        InitError(err);
        return 1;
    }
    uiInterface.InitMessage("Starting network threads...");
    if (!StartNetwork(*node, err)) {
        InitError(err);
        return 1;
    }
    if (!StartZMQ(*node, err)) {
        InitError(err);
        return 1;
    }
    // periodic flush + mempool expiry
    node->scheduler->ScheduleEvery(
        [] {
            if (Chainstate* cs = GetChainstate()) {
                CValidationState st;
                cs->FlushStateToDisk(st, FLUSH_STATE_PERIODIC);
            }
        },
        60 * 1000);
    // -blocknotify (reference init.cpp BlockNotifyCallback): %s = new tip hash
    if (gArgs.IsArgSet("-blocknotify"))
        uiInterface.NotifyBlockTip.connect([](bool ibd, const CBlockIndex* tip) {
            if (ibd || !tip) return;
            std::string cmd = gArgs.GetArg("-blocknotify", "");
            ReplaceAll(cmd, "%s", tip->GetBlockHash().GetHex());
            RunCommandAsync(cmd);
        });
    SetRPCWarmupFinished();
    uiInterface.InitMessage("Done loading");

    while (!g_signalled.load() && !ShutdownRequested()) MilliSleep(200);

    // ---- shutdown (reference init.cpp Shutdown(): RPC, network, wallet, mempool dump, flush)
    LogPrintf("Shutdown: In progress...\n");
    if (importThread.joinable()) importThread.join();
    uiInterface.NotifyBlockTip.disconnect_all();
    if (http) http->Stop();
    StopHTTPRPC(datadir);
    StopZMQ(*node);
    StopNetwork(*node);
    if (gArgs.GetBoolArg("-persistmempool", true)) node->chainstate->DumpMempool(datadir + "/mempool.dat");
    if (node->mempool && node->mempool->Estimator()) node->mempool->Estimator()->Write(datadir + "/fee_estimates.dat");
    StopWallet(*node);
    if (node->scheduler) node->scheduler->Stop();
    node->chainstate->Shutdown();
    // join the GPU verification lanes and destroy their HIP streams now, while the HIP runtime is
    // still up (the static singleton's destructor would run after it is torn down)
    GpuVerifyService::Instance().Shutdown();
    SetChainstate(nullptr);
    SetNode(nullptr);
    RemoveFile(datadir + "/" + gArgs.GetArg("-pid", "bitcoincashplusd.pid"));
    LogPrintf("Shutdown: done\n");
    LogShutdown();
    return 0;
}

} // namespace bcp
