// bench_bcp: native micro-benchmark harness.
// Parity: reference src/bench/ (bench.{h,cpp} adaptive State::KeepRunning with min/max/
// median per-iteration timing, -filter regex, CSV-like output; benches Sleep100ms, Trig,
// Base58Encode/CheckEncode/Decode, CCoinsCaching, DeserializeBlockTest,
// DeserializeAndCheckBlockTest (bench/data/block413567.raw, legacy header format),
// CCheckQueueSpeed, CoinSelection, RIPEMD160, SHA1, SHA256, SHA512, SHA256_32b,
// SipHash_32b, FastRandom_32bit/1bit, LockedPool, MempoolEviction, RollingBloom) plus
// MI355X batches (SHA256d64 batch, Merkle root, ECDSA batch verify) when a GPU is visible.
#include <unistd.h>
#include "consensus/merkle.h"
#include "consensus/tx_verify.h"
#include "consensus/merkleblock.h"
#include "consensus/params.h"
#include "crypto/hashes.h"
#include "kernels/gpu_api.h"
#include "keys/key.h"
#include "node/coins.h"
#include "node/kvstore.h"
#include "node/miner.h"
#include "script/sign.h"
#include "script/standard.h"
#include "node/sigverify.h"
#include "node/gpuverify.h"
#include "consensus/pow.h"
#include "consensus/equihash.h"
#include "secp256k1/secp256k1.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "primitives/block.h"
#include "util/lockedpool.h"
#include "util/strencodings.h"
#include "util/util.h"
#include "wallet/wallet.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <functional>
#include <regex>
#include <thread>

using namespace bcp;

namespace bench {

class State {
public:
    State(const std::string& name, double minTime) : name(name), minTime(minTime) {}
    bool KeepRunning() {
        const auto now = std::chrono::steady_clock::now();
        if (count == 0) {
            start = last = now;
            count = 1;
            return true;
        }
        const double dt = std::chrono::duration<double>(now - last).count();
        samples.push_back(dt);
        last = now;
        count++;
        const double elapsed = std::chrono::duration<double>(now - start).count();
        return elapsed < minTime && count < 1000000000ULL;
    }
    void Report() const {
        if (samples.empty()) return;
        std::vector<double> s = samples;
        std::sort(s.begin(), s.end());
        double total = 0;
        for (double d : s) total += d;
        // quartiles for the spread (IQR = p75 - p25)
        printf("%-34s %10zu %14.9f %14.9f %14.9f %14.9f %14.9f %14.9f\n", name.c_str(), s.size(), total, s.front(),
               s.back(), s[s.size() / 2], s[s.size() / 4], s[(3 * s.size()) / 4]);
        fflush(stdout);
    }

private:
    std::string name;
    double minTime;
    uint64_t count = 0;
    std::chrono::steady_clock::time_point start, last;
    std::vector<double> samples;
};

typedef std::function<void(State&)> BenchFn;
std::vector<std::pair<std::string, BenchFn>>& Registry() {
    static std::vector<std::pair<std::string, BenchFn>> r;
    return r;
}
struct Reg {
    Reg(const char* n, BenchFn f) { Registry().push_back({n, f}); }
};
#define BENCHMARK(fn) static bench::Reg reg_##fn(#fn, fn)

} // namespace bench
using bench::State;

static std::string g_dataDir = "bench/data";

// ------------------------------------------------------------------ benches
static void Sleep100ms(State& st) {
    while (st.KeepRunning()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
}
BENCHMARK(Sleep100ms);

static void Trig(State& st) {
    double sum = 0, d = 0.01;
    while (st.KeepRunning()) {
        sum += sin(d);
        d += 0.000001;
    }
    if (sum == 42) printf("x");
}
BENCHMARK(Trig);

static void Base58Encode(State& st) {
    unsigned char buf[32] = {17, 79, 8, 99, 150, 189, 208, 162, 22, 23, 203, 163, 36, 58, 147, 227,
                             139, 2, 215, 100, 91, 38, 11, 141, 253, 40, 117, 21, 16, 90, 200, 24};
    while (st.KeepRunning()) EncodeBase58(buf, buf + 32);
}
BENCHMARK(Base58Encode);

static void Base58CheckEncode(State& st) {
    std::vector<unsigned char> v(32, 7);
    while (st.KeepRunning()) EncodeBase58Check(v);
}
BENCHMARK(Base58CheckEncode);

static void Base58Decode(State& st) {
    const std::string addr = "17VZNX1SN5NtKa8UQFxwQbFeFc3iqRYhem";
    std::vector<unsigned char> v;
    while (st.KeepRunning()) DecodeBase58(addr, v);
}
BENCHMARK(Base58Decode);

static void HashBench(State& st, int which) {
    std::vector<unsigned char> in(1000 * 1000, 0);
    unsigned char out[64];
    while (st.KeepRunning()) {
        switch (which) {
        case 0: CRIPEMD160().Write(in.data(), in.size()).Finalize(out); break;
        case 1: CSHA1().Write(in.data(), in.size()).Finalize(out); break;
        case 2: CSHA256().Write(in.data(), in.size()).Finalize(out); break;
        case 3: CSHA512().Write(in.data(), in.size()).Finalize(out); break;
        }
    }
}
static void RIPEMD160(State& st) { HashBench(st, 0); }
static void SHA1(State& st) { HashBench(st, 1); }
static void SHA256(State& st) { HashBench(st, 2); }
static void SHA512(State& st) { HashBench(st, 3); }
BENCHMARK(RIPEMD160);
BENCHMARK(SHA1);
BENCHMARK(SHA256);
BENCHMARK(SHA512);

static void SHA256_32b(State& st) {
    std::vector<unsigned char> in(32, 0);
    while (st.KeepRunning())
        for (int i = 0; i < 1000000; i++) CSHA256().Write(in.data(), in.size()).Finalize(in.data());
}
BENCHMARK(SHA256_32b);

static void SipHash_32b(State& st) {
    uint256 x;
    uint64_t k1 = 0;
    while (st.KeepRunning())
        for (int i = 0; i < 1000000; i++) *((uint64_t*)x.begin()) = SipHashUint256(0, ++k1, x.begin());
}
BENCHMARK(SipHash_32b);

// One CPU ECDSA verification (CPubKey::Verify path: DER parse, key parse, GLV ecmult) per
// iteration, and the double-scalar multiplication alone with and without the endomorphism.
static void ECDSAVerify_CPU(State& st) {
    CKey key;
    key.MakeNewKey(true);
    uint256 h;
    Sha256d((const unsigned char*)"bench", 5, h.begin());
    std::vector<unsigned char> sig;
    key.Sign(h, sig);
    const std::vector<unsigned char> pub = key.GetPubKey().Raw();
    while (st.KeepRunning())
        if (!secp::VerifySignature(pub.data(), pub.size(), sig.data(), sig.size(), h.begin())) abort();
}
BENCHMARK(ECDSAVerify_CPU);
static void EcmultVariant(State& st, bool glv) {
    secp::Scalar na, ng, ka;
    unsigned char b[32];
    for (int i = 0; i < 32; i++) b[i] = (unsigned char)(i * 37 + 1);
    secp::sc_set_b32(na, b);
    for (int i = 0; i < 32; i++) b[i] = (unsigned char)(i * 11 + 5);
    secp::sc_set_b32(ng, b);
    for (int i = 0; i < 32; i++) b[i] = (unsigned char)(i * 7 + 3);
    secp::sc_set_b32(ka, b);
    secp::Gej A, r;
    secp::ecmult_gen(A, ka);
    while (st.KeepRunning()) {
        if (glv) secp::ecmult(r, A, na, ng);
        else secp::ecmult_plain(r, A, na, ng);
    }
}
static bench::Reg reg_EcmultGLV("Ecmult_CPU_GLV", [](State& st) { EcmultVariant(st, true); });
static bench::Reg reg_EcmultPlain("Ecmult_CPU_Plain", [](State& st) { EcmultVariant(st, false); });

static void FastRandom_32bit(State& st) {
    FastRandomContext rng(true);
    uint32_t x = 0;
    while (st.KeepRunning())
        for (int i = 0; i < 1000000; i++) x += (uint32_t)rng.randbits(32);
    if (x == 42) printf("x");
}
BENCHMARK(FastRandom_32bit);

static void FastRandom_1bit(State& st) {
    FastRandomContext rng(true);
    uint32_t x = 0;
    while (st.KeepRunning())
        for (int i = 0; i < 1000000; i++) x += (uint32_t)rng.randbits(1);
    if (x == 42) printf("x");
}
BENCHMARK(FastRandom_1bit);

static void RollingBloom(State& st) {
    CRollingBloomFilter filter(120000, 0.000001);
    std::vector<unsigned char> data(32);
    uint32_t count = 0;
    while (st.KeepRunning()) {
        count++;
        memcpy(data.data(), &count, 4);
        filter.insert(data);
        data[0] ^= 0xff;
        filter.contains(data);
    }
}
BENCHMARK(RollingBloom);

static void LockedPoolBench(State& st) {
    void* synth_base = reinterpret_cast<void*>(0x08000000);
    const size_t synth_size = 1024 * 1024;
    Arena b(synth_base, synth_size, 16);
    std::vector<void*> addr(128, nullptr);
    uint32_t s = 0x12345678;
    while (st.KeepRunning()) {
        for (int x = 0; x < 1000; ++x) {
            const int idx = s & (addr.size() - 1);
            if (s & 0x80000000) {
                b.free(addr[idx]);
                addr[idx] = nullptr;
            } else if (!addr[idx]) {
                addr[idx] = b.alloc((s >> 16) & 2047);
            }
            const bool lsb = s & 1;
            s >>= 1;
            if (lsb) s ^= 0xf00f00f0;
        }
    }
    for (void* p : addr) b.free(p);
}
static bench::Reg reg_LockedPool("LockedPool", LockedPoolBench);

static std::vector<unsigned char> LoadBlockFile() {
    std::ifstream f(g_dataDir + "/block413567.raw", std::ios::binary);
    return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static void DeserializeBlockTest(State& st) {
    const std::vector<unsigned char> raw = LoadBlockFile();
    if (raw.empty()) return;
    while (st.KeepRunning()) {
        CBlock block;
        SpanReader r(raw.data(), raw.size(), SER_NETWORK, PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY);
        r >> block;
    }
}
BENCHMARK(DeserializeBlockTest);

static void DeserializeAndCheckBlockTest(State& st) {
    const std::vector<unsigned char> raw = LoadBlockFile();
    if (raw.empty()) return;
    SelectParams("main");
    ChainstateOptions o;
    o.memoryOnly = true;
    o.useGpu = false;
    Chainstate cs(Params(), o);
    while (st.KeepRunning()) {
        CBlock block;
        SpanReader r(raw.data(), raw.size(), SER_NETWORK, PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY);
        r >> block;
        CValidationState state;
        if (!cs.CheckBlock(block, state)) {
            fprintf(stderr, "CheckBlock failed: %s\n", state.GetRejectReason().c_str());
            exit(1);
        }
    }
}
BENCHMARK(DeserializeAndCheckBlockTest);

static void CCheckQueueSpeed(State& st) {
    // 128 batches of trivial jobs through the worker pool (reference: prevector-free jobs)
    WorkerPool pool(std::max(2, GetNumCores()));
    std::atomic<uint64_t> sink{0};
    while (st.KeepRunning()) pool.ParallelFor(128 * 30, [&](size_t i) { sink += i; }, 30);
}
BENCHMARK(CCheckQueueSpeed);

static void CCoinsCaching(State& st) {
    CCoinsView base;
    CCoinsViewCache coins(&base);
    CBasicKeyStore ks;
    CKey key;
    key.MakeNewKey(true);
    ks.AddKey(key);
    CMutableTransaction prev;
    prev.vout.resize(2);
    prev.vout[0] = CTxOut(21 * 100000000LL, GetScriptForDestination(key.GetPubKey().GetID()));
    prev.vout[1] = CTxOut(22 * 100000000LL, GetScriptForDestination(key.GetPubKey().GetID()));
    const CTransaction prevTx(prev);
    AddCoins(coins, prevTx, 0);
    CMutableTransaction t;
    t.vin.resize(2);
    t.vin[0].prevout = COutPoint(prevTx.GetHash(), 0);
    t.vin[1].prevout = COutPoint(prevTx.GetHash(), 1);
    t.vout.resize(1);
    t.vout[0].nValue = 90 * 100000000LL;
    const CTransaction tx(t);
    while (st.KeepRunning()) {
        bool ok = true;
        for (const CTxIn& in : tx.vin) ok &= coins.HaveCoin(in.prevout);
        Amount v = 0;
        for (const CTxIn& in : tx.vin) v += coins.AccessCoin(in.prevout).out.nValue;
        if (!ok || v == 0) exit(1);
    }
}
BENCHMARK(CCoinsCaching);

// The view updates of one 8 MB block's UTXO pass, alone: 42k spends of fetched coins and 42k
// new P2PKH outputs into a fresh per-block cache sized up front (the serial tail of the parallel
// pass in ConnectBlockPrepare)
static void CoinsApply84k(State& st) {
    CCoinsView base;
    const size_t N = 42000;
    std::vector<COutPoint> spent(N), made(N);
    FastRandomContext rng(true);
    for (size_t i = 0; i < N; i++) {
        spent[i] = COutPoint(rng.rand256(), (uint32_t)(i & 1));
        made[i] = COutPoint(rng.rand256(), (uint32_t)(i & 1));
    }
    const CScript spk = CScript() << OP_DUP << OP_HASH160 << std::vector<unsigned char>(20, 7) << OP_EQUALVERIFY
                                  << OP_CHECKSIG;
    while (st.KeepRunning()) {
        CCoinsViewCache view(&base);
        view.Reserve(2 * N);
        for (size_t i = 0; i < N; i++) view.SpendFetchedMoved(spent[i]);
        for (size_t i = 0; i < N; i++) view.AddCoin(made[i], Coin(CTxOut(1000, spk), 100, false), false);
    }
}
BENCHMARK(CoinsApply84k);

// The same updates one coins-map shard per pool task (the parallel UTXO pass's view updates)
static void CoinsApply84k_Sharded(State& st) {
    CCoinsView base;
    const size_t N = 42000;
    std::vector<COutPoint> spent(N), made(N);
    FastRandomContext rng(true);
    for (size_t i = 0; i < N; i++) {
        spent[i] = COutPoint(rng.rand256(), (uint32_t)(i & 1));
        made[i] = COutPoint(rng.rand256(), (uint32_t)(i & 1));
    }
    std::vector<uint8_t> ss(N), ms(N);
    for (size_t i = 0; i < N; i++) {
        ss[i] = (uint8_t)CCoinsMap::ShardOf(spent[i]);
        ms[i] = (uint8_t)CCoinsMap::ShardOf(made[i]);
    }
    const CScript spk = CScript() << OP_DUP << OP_HASH160 << std::vector<unsigned char>(20, 7) << OP_EQUALVERIFY
                                  << OP_CHECKSIG;
    WorkerPool pool(std::min(16, std::max(2, GetNumCores())));
    while (st.KeepRunning()) {
        CCoinsViewCache view(&base);
        view.Reserve(2 * N);
        view.ForEachShard(
            [&](unsigned sh) {
                for (size_t i = 0; i < N; i++)
                    if (ss[i] == sh) view.SpendFetchedMoved(spent[i]);
                for (size_t i = 0; i < N; i++)
                    if (ms[i] == sh) view.AddCoin(made[i], Coin(CTxOut(1000, spk), 100, false), false);
            },
            &pool);
    }
}
BENCHMARK(CoinsApply84k_Sharded);

// One block's updates applied to a large coins tip in place (ConnectTip's parallel UTXO pass):
// 42k spends of the previous block's outputs (FRESH entries, erased) and 42k new outputs, one
// shard per pool task, on a tip that already holds -tipcoins entries (default 400k)
static void CoinsTipApply84k_Sharded(State& st) {
    CCoinsView base;
    CCoinsViewCache tip(&base);
    const size_t N = 42000, held = (size_t)gArgs.GetArg("-tipcoins", (int64_t)400000);
    FastRandomContext rng(true);
    const CScript spk = CScript() << OP_DUP << OP_HASH160 << std::vector<unsigned char>(20, 7) << OP_EQUALVERIFY
                                  << OP_CHECKSIG;
    for (size_t i = 0; i < held; i++) tip.AddCoin(COutPoint(rng.rand256(), 0), Coin(CTxOut(1000, spk), 1, false), false);
    std::vector<COutPoint> prev(N);
    for (size_t i = 0; i < N; i++) {
        prev[i] = COutPoint(rng.rand256(), (uint32_t)(i & 1));
        tip.AddCoin(prev[i], Coin(CTxOut(1000, spk), 2, false), false);
    }
    WorkerPool pool(std::min(16, std::max(2, GetNumCores())));
    while (st.KeepRunning()) {
        std::vector<COutPoint> made(N);
        for (size_t i = 0; i < N; i++) made[i] = COutPoint(rng.rand256(), (uint32_t)(i & 1));
        std::vector<uint8_t> ss(N), ms(N);
        for (size_t i = 0; i < N; i++) {
            ss[i] = (uint8_t)CCoinsMap::ShardOf(prev[i]);
            ms[i] = (uint8_t)CCoinsMap::ShardOf(made[i]);
        }
        const int64_t t0 = GetTimeMicros();
        tip.ForEachShard(
            [&](unsigned sh) {
                for (size_t i = 0; i < N; i++)
                    if (ss[i] == sh) tip.SpendPeeked(prev[i]);
                for (size_t i = 0; i < N; i++)
                    if (ms[i] == sh) tip.AddCoin(made[i], Coin(CTxOut(1000, spk), 3, false), false);
            },
            &pool);
        fprintf(stderr, "# tip apply %.2f ms (tip %u entries)\n", (GetTimeMicros() - t0) / 1000.0, tip.GetCacheSize());
        prev.swap(made);
    }
}
BENCHMARK(CoinsTipApply84k_Sharded);

static void CoinSelection(State& st) {
    SelectParams("regtest");
    CWallet wallet("bench", "", true);
    std::vector<COutput> vCoins;
    std::vector<std::unique_ptr<CWalletTx>> wtxs;
    auto addCoin = [&](Amount nValue) {
        CMutableTransaction tx;
        tx.nLockTime = (uint32_t)wtxs.size();
        tx.vout.resize(1);
        tx.vout[0].nValue = nValue;
        wtxs.emplace_back(new CWalletTx(&wallet, MakeTransactionRef(std::move(tx))));
        wtxs.back()->fFromMe = true;
        vCoins.push_back({wtxs.back().get(), 0, 6 * 24, true, true});
    };
    for (int i = 0; i < 1000; i++) addCoin(1000 * 100000000LL);
    addCoin(3 * 100000000LL);
    while (st.KeepRunning()) {
        std::set<std::pair<const CWalletTx*, unsigned int>> setCoinsRet;
        Amount nValueRet;
        const bool ok = wallet.SelectCoinsMinConf(1003 * 100000000LL, 1, 6, 0, vCoins, setCoinsRet, nValueRet);
        if (!ok || nValueRet != 1003 * 100000000LL || setCoinsRet.size() != 2) exit(1);
    }
}
BENCHMARK(CoinSelection);

// ------------------------------------------------------------------ storage engine
// KVStoreCoins: the chainstate store at UTXO-set scale (VERDICT r2 "bounded-memory storage
// engine"). Inserts -kvcoins synthetic coins (key 'C' + 32-byte txid + vout varint, 30-45 byte
// values, the shape CCoinsViewDB writes) in 16 MB batches like CCoinsViewDB::BatchWrite, with the
// store sized from -kvdbcache exactly as the node sizes its coins store; then random reads of
// present and absent keys and one full ordered scan. Reports peak RSS against -kvdbcache + 200 MB.
static size_t RssKB(const char* field) {
    FILE* f = fopen("/proc/self/status", "r");
    if (!f) return 0;
    char line[256];
    size_t kb = 0;
    while (fgets(line, sizeof(line), f))
        if (strncmp(line, field, strlen(field)) == 0) kb = (size_t)strtoull(line + strlen(field), nullptr, 10);
    fclose(f);
    return kb;
}
static uint64_t Mix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
static std::string CoinKeyOf(uint64_t i, bool present = true) {
    std::string k(1, 'C');
    const uint64_t t = i / 3; // three outputs per synthetic txid
    for (int w = 0; w < 4; w++) {
        const uint64_t v = Mix64(t * 4 + w + (present ? 0 : 0x5555555555555555ull));
        k.append((const char*)&v, 8);
    }
    k.push_back((char)(i % 3));
    return k;
}
static void KVStoreCoins(State& st) {
    const uint64_t n = (uint64_t)gArgs.GetArg("-kvcoins", (int64_t)50000000);
    const size_t dbcache = (size_t)gArgs.GetArg("-kvdbcache", (int64_t)450) << 20;
    const size_t coinDBCache = std::min(dbcache / 2, dbcache / 4 + ((size_t)1 << 23));
    KVOptions o;
    o.memtableBytes = std::max<size_t>(coinDBCache / 4, 1u << 20);
    o.blockCacheBytes = coinDBCache / 2;
    char tmpl[] = "/tmp/bcp_kvbench_XXXXXX";
    const std::string dir = std::string(mkdtemp(tmpl)) + "/chainstate";
    while (st.KeepRunning()) {
        const size_t rss0 = RssKB("VmRSS:");
        const auto t0 = std::chrono::steady_clock::now();
        KVStore db(dir, false, true, o);
        KVBatch b;
        std::string val;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t r = Mix64(i ^ 0xabcdefull);
            val.assign(30 + (size_t)(r % 16), (char)(r >> 8));
            b.WriteRaw(CoinKeyOf(i), val);
            if (b.SizeEstimate() > (16u << 20)) db.WriteBatch(b);
            if ((i & ((1u << 22) - 1)) == 0 && i)
                fprintf(stderr, "  kv: %llu coins, rss %zu MB, %zu segments\n", (unsigned long long)i,
                        RssKB("VmRSS:") >> 10, db.Stats().segments);
        }
        db.WriteBatch(b, true);
        db.Flush();
        const auto t1 = std::chrono::steady_clock::now();
        FastRandomContext rng(true);
        std::string v;
        const int reads = 1000000;
        size_t found = 0;
        for (int i = 0; i < reads; i++) found += db.ReadRaw(CoinKeyOf(rng.randrange(n)), v) ? 1 : 0;
        const auto t2 = std::chrono::steady_clock::now();
        size_t absent = 0;
        for (int i = 0; i < reads; i++) absent += db.ReadRaw(CoinKeyOf(rng.randrange(n), false), v) ? 0 : 1;
        const auto t3 = std::chrono::steady_clock::now();
        uint64_t scanned = 0;
        auto it = db.NewIterator();
        for (it->Seek(std::string(1, 'C')); it->Valid(); it->Next()) ++scanned;
        const auto t4 = std::chrono::steady_clock::now();
        const KVStats s = db.Stats();
        const size_t peak = RssKB("VmHWM:");
        auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
            return std::chrono::duration<double>(z - a).count();
        };
        printf("{\"bench\": \"KVStoreCoins\", \"coins\": %llu, \"dbcache_mb\": %zu, \"insert_s\": %.2f, "
               "\"insert_per_s\": %.0f, \"read_hit_us\": %.2f, \"read_miss_us\": %.2f, \"hits\": %zu, "
               "\"misses_absent\": %zu, \"scan_s\": %.2f, \"scanned\": %llu, \"segments\": %zu, \"disk_mb\": %.0f, "
               "\"index_mb\": %.1f, \"bloom_mb\": %.1f, \"flushes\": %llu, \"merges\": %llu, \"stalls\": %llu, "
               "\"rss_start_mb\": %zu, \"rss_peak_mb\": %zu, \"budget_mb\": %zu, \"within_budget\": %s}\n",
               (unsigned long long)n, dbcache >> 20, sec(t0, t1), n / sec(t0, t1), sec(t1, t2) * 1e6 / reads,
               sec(t2, t3) * 1e6 / reads, found, absent, sec(t3, t4), (unsigned long long)scanned, s.segments,
               s.segmentBytes / 1048576.0, s.indexBytes / 1048576.0, s.bloomBytes / 1048576.0,
               (unsigned long long)s.flushes, (unsigned long long)s.merges, (unsigned long long)s.stalls, rss0 >> 10,
               peak >> 10, (dbcache >> 20) + 200 + (rss0 >> 10), peak <= rss0 + ((dbcache + (200u << 20)) >> 10) ? "true" : "false");
        fflush(stdout);
    }
    const std::string cmd = "rm -rf '" + dir.substr(0, dir.rfind('/')) + "'";
    if (system(cmd.c_str()) != 0) {}
}
BENCHMARK(KVStoreCoins);

static void MempoolEviction(State& st) {
    CTxMemPool pool(nullptr);
    std::vector<CTransactionRef> txs;
    for (int i = 0; i < 7; i++) {
        CMutableTransaction tx;
        tx.vin.resize(1);
        tx.vin[0].prevout = COutPoint(uint256S(strprintf("%064x", i + 1)), 0);
        tx.vin[0].scriptSig = CScript() << OP_1;
        tx.vout.resize(1);
        tx.vout[0].scriptPubKey = CScript() << OP_1 << OP_EQUAL;
        tx.vout[0].nValue = 10 * 100000000LL;
        txs.push_back(MakeTransactionRef(std::move(tx)));
    }
    while (st.KeepRunning()) {
        int64_t t = 0;
        for (size_t i = 0; i < txs.size(); i++) {
            CTxMemPoolEntry e(txs[i], (Amount)(1000 * (i + 1)), t++, 0.0, 1, 0, false, 1, LockPoints());
            pool.addUnchecked(txs[i]->GetHash(), e);
        }
        pool.TrimToSize(pool.DynamicMemoryUsage() * 3 / 4);
        pool.TrimToSize(GetSerializeSize(*txs[0]));
        pool.clear();
    }
}
BENCHMARK(MempoolEviction);

// ---- MI355X batches (skipped without a GPU)
static void GpuSha256d64Batch(State& st) {
    if (!gpu::GpuAvailable()) return;
    std::vector<unsigned char> data(64 * (1 << 20), 1);
    while (st.KeepRunning()) gpu::Sha256d64Batch(data);
}
static bench::Reg reg_GpuSha("GPU_SHA256d64_1M", GpuSha256d64Batch);

static void GpuMerkle(State& st) {
    if (!gpu::GpuAvailable()) return;
    std::vector<unsigned char> leaves(32 * (1 << 20), 3);
    bool mut = false;
    while (st.KeepRunning()) gpu::MerkleRoot(leaves, &mut);
}
static bench::Reg reg_GpuMerkle("GPU_MerkleRoot_1M", GpuMerkle);

// Merkle roots at the sizes of real blocks: ~21k transactions fill 8 MB with 2-in/2-out P2PKH
// spends; 1M leaves bound the largest block.
static void MerkleBench(State& st, size_t n, bool gpuPath) {
    if (gpuPath && !gpu::GpuAvailable()) return;
    std::vector<unsigned char> leaves(32 * n);
    for (size_t i = 0; i < leaves.size(); i++) leaves[i] = (unsigned char)(i * 131 + 7);
    std::vector<uint256> v(n);
    for (size_t i = 0; i < n; i++) memcpy(v[i].begin(), leaves.data() + 32 * i, 32);
    while (st.KeepRunning()) {
        bool mut = false;
        if (gpuPath) gpu::MerkleRoot(leaves, &mut);
        else ComputeMerkleRoot(v, &mut);
    }
}
static bench::Reg reg_GpuMerkle21k("GPU_MerkleRoot_21k", [](State& st) { MerkleBench(st, 21001, true); });
static bench::Reg reg_CpuMerkle21k("CPU_MerkleRoot_21k", [](State& st) { MerkleBench(st, 21001, false); });

static void CpuSha256d64(State& st) {
    std::vector<unsigned char> data(64 * (1 << 20), 1), out(32 * (1 << 20));
    while (st.KeepRunning()) Sha256d64(out.data(), data.data(), 1u << 20);
}
static bench::Reg reg_CpuSha("CPU_SHA256d64_1M", CpuSha256d64);

static void CpuMerkle(State& st) {
    std::vector<uint256> leaves(1 << 20);
    for (size_t i = 0; i < leaves.size(); i++) *(uint64_t*)leaves[i].begin() = i;
    while (st.KeepRunning()) {
        bool mut = false;
        ComputeMerkleRoot(leaves, &mut);
    }
}
static bench::Reg reg_CpuMerkle("CPU_MerkleRoot_1M", CpuMerkle);

// BIP152 short ids of a large mempool (K9): SipHash-2-4 of 250k txids, CPU loop vs GPU batch
// (incl. pinned staging and both copies).
static void ShortIdBench(State& st, bool gpuPath) {
    if (gpuPath && !gpu::GpuAvailable()) return;
    const size_t n = 250000;
    std::vector<unsigned char> ids(32 * n);
    for (size_t i = 0; i < ids.size(); i++) ids[i] = (unsigned char)(i * 2654435761u >> 13);
    std::vector<uint64_t> out(n);
    while (st.KeepRunning()) {
        if (gpuPath) out = gpu::ShortTxIdBatch(0x0706050403020100ULL, 0x0f0e0d0c0b0a0908ULL, ids.data(), n);
        else
            for (size_t i = 0; i < n; i++)
                out[i] = SipHashUint256(0x0706050403020100ULL, 0x0f0e0d0c0b0a0908ULL, &ids[32 * i]) & 0xffffffffffffULL;
    }
}
static bench::Reg reg_CpuShortId("CPU_ShortIds_250k", [](State& st) { ShortIdBench(st, false); });
static bench::Reg reg_GpuShortId("GPU_ShortIds_250k", [](State& st) { ShortIdBench(st, true); });

// ---- verify-service sharding overhead on one GPU: the same batch over lanes [0], [0,0] and
// [0,0,0,0] (one stream and one host-fill worker group each). 199k deferred ECDSA checks
// (1024 distinct signatures repeated, end to end from DeferredSigCheck records: DER parse, key
// forms, upload, prep + verify kernels, verdicts) and a 2000-header Equihash(200,9) batch
// (CheckEquihashSolutions: raw header bytes staged, BLAKE2b states and verification on the
// device; random solutions cost the kernel the same as valid ones).
static void LanesEcdsa(State& st, int lanes) {
    if (!gpu::GpuAvailable()) return;
    static std::vector<DeferredSigCheck> checks;
    if (checks.empty()) {
        std::vector<DeferredSigCheck> uniq(1024);
        for (size_t i = 0; i < uniq.size(); i++) {
            CKey key;
            key.MakeNewKey(true);
            uint256 h;
            Sha256d((const unsigned char*)&i, sizeof(i), h.begin());
            std::vector<unsigned char> sig;
            key.Sign(h, sig);
            uniq[i].sighash = h;
            uniq[i].sig.assign(sig);
            uniq[i].pubkey.assign(key.GetPubKey().Raw());
        }
        checks.resize(199000);
        for (size_t i = 0; i < checks.size(); i++) checks[i] = uniq[i % uniq.size()];
    }
    std::vector<const DeferredSigCheck*> ptrs(checks.size());
    for (size_t i = 0; i < checks.size(); i++) ptrs[i] = &checks[i];
    GpuVerifyService& svc = GpuVerifyService::Instance();
    svc.SetDevices(std::vector<int>(lanes, 0));
    svc.SetMinShard(1024, 64);
    std::vector<uint8_t> r = GpuVerifyDeferred(ptrs); // lanes up, buffers grown
    while (st.KeepRunning()) r = GpuVerifyDeferred(ptrs);
    if (std::count(r.begin(), r.end(), 1) != (long)r.size()) {
        fprintf(stderr, "LanesEcdsa: %zu of %zu verdicts false\n", (size_t)std::count(r.begin(), r.end(), 0), r.size());
        exit(1);
    }
    svc.SetMinShard(65536, 2048); // the service defaults
    svc.SetDevices({});
}
static bench::Reg reg_LanesEcdsa1("Lanes1_Ecdsa199k_GPU", [](State& st) { LanesEcdsa(st, 1); });
static bench::Reg reg_LanesEcdsa2("Lanes2_Ecdsa199k_GPU", [](State& st) { LanesEcdsa(st, 2); });
static bench::Reg reg_LanesEcdsa4("Lanes4_Ecdsa199k_GPU", [](State& st) { LanesEcdsa(st, 4); });

static void LanesHeaders(State& st, int lanes) {
    if (!gpu::GpuAvailable()) return;
    SelectParams("main");
    static std::vector<CBlockHeader> headers;
    if (headers.empty()) {
        FastRandomContext rng(true);
        headers.resize(2000);
        for (CBlockHeader& h : headers) {
            h.nVersion = 4;
            h.hashPrevBlock = rng.rand256();
            h.hashMerkleRoot = rng.rand256();
            h.nTime = 1500000000 + rng.rand32() % 1000000;
            h.nBits = 0x1d00ffff;
            h.nNonce = rng.rand256();
            h.nSolution.resize(1344);
            for (auto& b : h.nSolution) b = (unsigned char)rng.rand32();
        }
    }
    std::vector<const CBlockHeader*> ptrs;
    for (const CBlockHeader& h : headers) ptrs.push_back(&h);
    GpuVerifyService& svc = GpuVerifyService::Instance();
    svc.SetDevices(std::vector<int>(lanes, 0));
    svc.SetMinShard(1024, 64);
    std::vector<bool> r = CheckEquihashSolutions(ptrs, Params(), true);
    while (st.KeepRunning()) r = CheckEquihashSolutions(ptrs, Params(), true);
    svc.SetMinShard(65536, 2048); // the service defaults
    svc.SetDevices({});
}
static bench::Reg reg_LanesHdr1("Lanes1_Headers2000_GPU", [](State& st) { LanesHeaders(st, 1); });
static bench::Reg reg_LanesHdr2("Lanes2_Headers2000_GPU", [](State& st) { LanesHeaders(st, 2); });
static bench::Reg reg_LanesHdr4("Lanes4_Headers2000_GPU", [](State& st) { LanesHeaders(st, 4); });
// the same 2000 headers with host-built states (the round-3 path), for the prep split
static void HeadersHostStates(State& st) {
    if (!gpu::GpuAvailable()) return;
    SelectParams("main");
    const EquihashParams ep(200, 9);
    FastRandomContext rng(true);
    std::vector<CBlockHeader> headers(2000);
    for (CBlockHeader& h : headers) {
        h.nVersion = 4;
        h.hashPrevBlock = rng.rand256();
        h.nNonce = rng.rand256();
        h.nSolution.resize(1344);
        for (auto& b : h.nSolution) b = (unsigned char)rng.rand32();
    }
    while (st.KeepRunning()) {
        std::vector<gpu::EhBaseState> states;
        std::vector<const std::vector<unsigned char>*> sols;
        for (const CBlockHeader& h : headers) {
            CBlake2b b = EhInitialiseState(ep);
            std::vector<unsigned char> in = h.EquihashInput();
            b.Write(in.data(), in.size());
            b.Write(h.nNonce.begin(), 32);
            states.push_back(gpu::MakeEhBaseState(b));
            sols.push_back(&h.nSolution);
        }
        GpuVerifyService::Instance().Equihash(200, 9, states, sols);
    }
}
BENCHMARK(HeadersHostStates);

// ---- 8 MB block connect (BASELINE.md "block connect time for an 8 MB / 160k-sigop block"): a
// regtest chain past the BCP fork (Equihash(48,5) headers) in a memory-only chainstate, one big
// block on top of it, then Chainstate::TestBlockValidity (CheckBlock + contextual checks +
// ConnectBlock with every script and signature checked, nothing cached) per iteration. _GPU
// batches the ECDSA checks on the MI355X; _CPU keeps them on the worker pool.
//   ConnectBlock8MB:             21,000 2-in/2-out P2PKH transactions (42,000 FORKID signatures,
//                                7.83 MB), outputs P2PKH.
//   ConnectBlock8MB_160kSigops:  the consensus worst case of an 8 MB block: 19,500 2-in/2-out
//                                P2PKH transactions paying to P2SH (39,000 signatures, no sigops
//                                of their own) plus 8 transactions of 198 P2SH inputs whose redeem
//                                script is <pk> (2DUP CHECKSIGVERIFY) x100 CHECKSIG (201 ops, 101
//                                accurately counted sigops each): 159,984 sigops of the 160,000
//                                allowed (20,000 per started MB, reference src/consensus/consensus.h:
//                                115,137-140), 198,984 signature checks in 7.8 MB.
namespace {
struct BigBlockFixture {
    std::unique_ptr<Chainstate> cs;
    CTxMemPool pool;
    CBlock block;
    size_t nSigs = 0, nBytes = 0, nSigOps = 0;
    bool ok = false;
};

CBlock MakeBlock(Chainstate& cs, CTxMemPool& pool, const CScript& spk, const std::vector<CTransactionRef>& txs) {
    BlockAssembler::Options o;
    BlockAssembler ba(cs, &pool, o);
    std::unique_ptr<CBlockTemplate> t = ba.CreateNewBlock(spk);
    CBlock b = t->block;
    unsigned extra = 0;
    IncrementExtraNonce(&b, cs.Tip(), extra, cs.MaxBlockSize()); // BIP34 height in the coinbase
    for (const auto& tx : txs) b.vtx.push_back(tx);
    b.hashMerkleRoot = BlockMerkleRoot(b);
    uint64_t tries = 1u << 24;
    if (!SolveBlock(b, Params(), tries, false)) throw std::runtime_error("bench: SolveBlock failed");
    return b;
}

// kind 0: P2PKH spends; 1: the 160k-sigop worst case; 2: P2SH 2-of-3 multisig spends (every
// CHECKMULTISIG deferred speculatively into the batch: 4 (signature, key) pairs per input)
BigBlockFixture& BigBlock(int kind) {
    static BigBlockFixture fx[3];
    static bool built[3] = {false, false, false};
    const bool worstCase = kind == 1, multisig = kind == 2;
    BigBlockFixture& f = fx[kind];
    if (built[kind]) return f;
    built[kind] = true;
    SelectParams("regtest");
    ChainstateOptions o;
    o.memoryOnly = true;
    char tmpl[] = "/tmp/bench_bcp_XXXXXX"; // block/undo files of the fixture chain
    if (!mkdtemp(tmpl)) throw std::runtime_error("bench: mkdtemp failed");
    o.datadir = tmpl;
    o.useGpu = gpu::GpuAvailable();
    o.scriptThreads = (int)gArgs.GetArg("-par", (int64_t)std::min(16, std::max(2, GetNumCores())));
    o.parallelUtxoMinTx = (size_t)gArgs.GetArg("-parallelutxo", (int64_t)o.parallelUtxoMinTx);
    f.cs.reset(new Chainstate(Params(), o));
    std::string err;
    if (!f.cs->InitBlockIndex(err)) throw std::runtime_error("bench: " + err);
    f.cs->SetMempool(&f.pool);
    CBasicKeyStore ks;
    CKey key;
    key.MakeNewKey(true);
    ks.AddKey(key);
    const CScript spk = GetScriptForDestination(key.GetPubKey().GetID());
    const uint32_t hashType = SIGHASH_ALL | SIGHASH_FORKID;
    // the worst-case redeem script and its P2SH output script
    CScript redeem;
    const CPubKey pub = key.GetPubKey();
    redeem << std::vector<unsigned char>(pub.begin(), pub.end());
    for (int i = 0; i < 100; i++) redeem << OP_2DUP << OP_CHECKSIGVERIFY;
    redeem << OP_CHECKSIG;
    const CScript spkSH = GetScriptForDestination(CScriptID(redeem));
    // 2-of-3 multisig behind P2SH (bare multisig outputs would count 20 sigops each)
    CKey k2, k3;
    k2.MakeNewKey(true);
    k3.MakeNewKey(false);
    ks.AddKey(k2);
    ks.AddKey(k3);
    CScript redeemMS;
    redeemMS << 2 << std::vector<unsigned char>(pub.begin(), pub.end()) << k2.GetPubKey().Raw() << k3.GetPubKey().Raw()
             << 3 << OP_CHECKMULTISIG;
    ks.AddCScript(redeemMS);
    const CScript spkMS = GetScriptForDestination(CScriptID(redeemMS));
    const CScript& fanOut = multisig ? spkMS : spk;
    const int NFAN = 24, NOUT = 1750;              // 42,000 outputs to spend
    const int NTX = worstCase ? 19500 : multisig ? 10700 : 21000; // 2-in/2-out spends in the big block
    const int NSHTX = worstCase ? 8 : 0, NSHIN = 198; // P2SH spends: 198 x 101 sigops < 20,000 per tx
    const CScript& bigOut = worstCase ? spkSH : spk;
    std::vector<CTransactionRef> coinbases;
    auto connect = [&](const CBlock& b) {
        bool fNew = false;
        CValidationState st;
        if (!f.cs->ProcessNewBlock(std::make_shared<const CBlock>(b), true, &fNew, &st)) {
            fprintf(stderr, "height %d txs %zu size %zu cb-sigops %llu\n", f.cs->Height(), b.vtx.size(),
                    GetSerializeSize(b, PROTOCOL_VERSION), (unsigned long long)GetSigOpCountWithoutP2SH(*b.vtx[0]));
            throw std::runtime_error("bench: ProcessNewBlock: " + FormatStateMessage(st));
        }
    };
    // past the regtest fork height: post-fork blocks carry NULLFAIL, which lets block validation
    // defer every CHECKSIG into one batch (pre-fork scripts verify inline, reference semantics)
    const int forkHeight = Params().GetConsensus().BCPHeight;
    while (f.cs->Height() < forkHeight + 1) {
        CBlock b = MakeBlock(*f.cs, f.pool, spk, {});
        coinbases.push_back(b.vtx[0]);
        connect(b);
    }
    // fan-out: NFAN matured coinbases -> NFAN * NOUT P2PKH outputs (+ one coinbase -> P2SH outputs)
    std::vector<CTransactionRef> fan;
    for (int c = 0; c < NFAN; c++) {
        const CTransaction& cb = *coinbases[c];
        CMutableTransaction m;
        m.vin.resize(1);
        m.vin[0].prevout = COutPoint(cb.GetHash(), 0);
        const Amount each = (cb.vout[0].nValue - 100000) / NOUT;
        for (int k = 0; k < NOUT; k++) m.vout.push_back(CTxOut(each, fanOut));
        if (!SignSignature(ks, cb.vout[0].scriptPubKey, m, 0, cb.vout[0].nValue, hashType))
            throw std::runtime_error("bench: fan-out signing failed");
        fan.push_back(MakeTransactionRef(std::move(m)));
    }
    CTransactionRef shFan;
    if (NSHTX) {
        const CTransaction& cb = *coinbases[NFAN];
        CMutableTransaction m;
        m.vin.resize(1);
        m.vin[0].prevout = COutPoint(cb.GetHash(), 0);
        const Amount each = (cb.vout[0].nValue - 100000) / (NSHTX * NSHIN);
        for (int k = 0; k < NSHTX * NSHIN; k++) m.vout.push_back(CTxOut(each, spkSH));
        if (!SignSignature(ks, cb.vout[0].scriptPubKey, m, 0, cb.vout[0].nValue, hashType))
            throw std::runtime_error("bench: P2SH fan-out signing failed");
        shFan = MakeTransactionRef(std::move(m));
    }
    // 8 fan-out transactions per block: a P2PKH output is one sigop in 34 bytes, so an output-only
    // block would exceed the 20,000-sigops-per-MB budget
    for (int c0 = 0; c0 < NFAN; c0 += 8) {
        std::vector<CTransactionRef> v(fan.begin() + c0, fan.begin() + c0 + 8);
        if (c0 == 0 && shFan) v.push_back(shFan);
        connect(MakeBlock(*f.cs, f.pool, spk, v));
    }
    // the big block: NTX transactions, 2 inputs and 2 outputs each, signed on the worker pool
    std::vector<CMutableTransaction> txs(NTX);
    WorkerPool wp(std::min(16, std::max(2, GetNumCores())));
    std::atomic<bool> signFail{false};
    wp.ParallelFor(NTX, [&](size_t t) {
        CMutableTransaction& m = txs[t];
        Amount in = 0;
        for (int k = 0; k < 2; k++) {
            const size_t u = 2 * t + k;
            const CTransaction& ft = *fan[u / NOUT];
            m.vin.emplace_back();
            m.vin.back().prevout = COutPoint(ft.GetHash(), (uint32_t)(u % NOUT));
            in += ft.vout[u % NOUT].nValue;
        }
        m.vout.push_back(CTxOut(in / 2 - 500, bigOut));
        m.vout.push_back(CTxOut(in / 2 - 500, bigOut));
        for (int k = 0; k < 2; k++) {
            const size_t u = 2 * t + k;
            const CTxOut& prev = fan[u / NOUT]->vout[u % NOUT];
            if (!SignSignature(ks, prev.scriptPubKey, m, k, prev.nValue, hashType)) signFail = true;
        }
    }, 64);
    if (signFail) throw std::runtime_error("bench: signing failed");
    // the worst-case P2SH spends: scriptSig <sig> <redeem>, one signature checked 101 times
    std::vector<CMutableTransaction> shTxs(NSHTX);
    for (int t = 0; t < NSHTX; t++) {
        CMutableTransaction& m = shTxs[t];
        Amount in = 0;
        for (int k = 0; k < NSHIN; k++) {
            const uint32_t n = (uint32_t)(t * NSHIN + k);
            m.vin.emplace_back();
            m.vin.back().prevout = COutPoint(shFan->GetHash(), n);
            in += shFan->vout[n].nValue;
        }
        m.vout.push_back(CTxOut(in - 10000, spkSH));
        const CTransaction unsigned_tx(m);
        const PrecomputedTransactionData txdata(unsigned_tx);
        for (int k = 0; k < NSHIN; k++) {
            const uint256 h = SignatureHash(redeem, unsigned_tx, k, hashType, shFan->vout[t * NSHIN + k].nValue,
                                            &txdata);
            std::vector<unsigned char> sig;
            if (!key.Sign(h, sig)) throw std::runtime_error("bench: P2SH signing failed");
            sig.push_back((unsigned char)hashType);
            m.vin[k].scriptSig = CScript() << sig << std::vector<unsigned char>(redeem.begin(), redeem.end());
        }
    }
    std::vector<CTransactionRef> refs;
    for (auto& m : txs) refs.push_back(MakeTransactionRef(std::move(m)));
    for (auto& m : shTxs) refs.push_back(MakeTransactionRef(std::move(m)));
    f.block = MakeBlock(*f.cs, f.pool, spk, refs);
    f.nSigs = (multisig ? 4 : 2) * (size_t)NTX + (size_t)NSHTX * NSHIN * 101;
    f.nBytes = GetSerializeSize(f.block, PROTOCOL_VERSION);
    {
        const CCoinsViewCache& view = f.cs->CoinsTip();
        for (const auto& tx : f.block.vtx)
            f.nSigOps += GetSigOpCountWithoutP2SH(*tx) + (tx->IsCoinBase() ? 0 : GetP2SHSigOpCount(*tx, view));
    }
    f.ok = true;
    fprintf(stderr, "# big block%s: %zu txs, %zu signature checks, %zu sigops (limit %llu), %zu bytes, on height %d\n",
            worstCase ? " (160k sigops)" : multisig ? " (2-of-3 P2SH multisig)" : "", f.block.vtx.size(), f.nSigs, f.nSigOps,
            (unsigned long long)GetMaxBlockSigOpsCount(f.nBytes), f.nBytes, f.cs->Height());
    return f;
}

void ConnectBigBlock(State& st, bool useGpu, int kind) {
    BigBlockFixture& f = BigBlock(kind);
    const size_t thr = GetGpuSigThreshold();
    SetGpuSigThreshold(useGpu ? DEFAULT_GPU_SIG_THRESHOLD : SIZE_MAX);
    const SigVerifyStats s0 = GetSigVerifyStats();
    int64_t ph0[Chainstate::PH_COUNT];
    for (int k = 0; k < Chainstate::PH_COUNT; k++) ph0[k] = f.cs->ConnectPhaseMicros((Chainstate::ConnectPhase)k);
    // -ecdsaminshard=N: a batch is split over the verify lanes only in shards of at least N
    if (gArgs.IsArgSet("-ecdsaminshard"))
        GpuVerifyService::Instance().SetMinShard((size_t)gArgs.GetArg("-ecdsaminshard", (int64_t)256), 32);
    auto laneTimes = [] {
        uint64_t fill = 0, dev = 0;
        for (const auto& L : GpuVerifyService::Instance().Stats()) {
            fill += L.fillMicros;
            dev += L.deviceMicros;
        }
        return std::make_pair(fill, dev);
    };
    const auto lt0 = laneTimes();
    int iters = 0;
    while (st.KeepRunning()) {
        CValidationState state;
        if (!f.cs->TestBlockValidity(state, f.block, f.cs->Tip(), false, true)) {
            fprintf(stderr, "TestBlockValidity failed: %s\n", state.GetRejectReason().c_str());
            exit(1);
        }
        iters++;
    }
    const SigVerifyStats s1 = GetSigVerifyStats();
    // where the time goes: signature batches (GPU incl. host DER parse/upload, or CPU pool)
    fprintf(stderr, "# %s: per block %.1f sigs on the GPU (%.2f ms), %.1f on the CPU (%.2f ms), %llu GPU failures, "
                    "%.1f deferred multisig groups\n",
            useGpu ? "GPU" : "CPU", (double)(s1.gpu_sigs - s0.gpu_sigs) / iters, (s1.gpu_ms - s0.gpu_ms) / iters,
            (double)(s1.cpu_sigs - s0.cpu_sigs) / iters, (s1.cpu_ms - s0.cpu_ms) / iters,
            (unsigned long long)(s1.gpu_failures - s0.gpu_failures),
            (double)(s1.multisig_groups - s0.multisig_groups) / iters);
    auto ms = [&](Chainstate::ConnectPhase k) { return 0.001 * (f.cs->ConnectPhaseMicros(k) - ph0[k]) / iters; };
    if (useGpu) {
        const auto lt1 = laneTimes();
        fprintf(stderr, "# GPU: verify lanes (ms/block, summed over lanes): host fill %.2f, device (copies + kernels) %.2f\n",
                0.001 * (lt1.first - lt0.first) / iters, 0.001 * (lt1.second - lt0.second) / iters);
    }
    fprintf(stderr, "# %s: connect phases (ms/block): checkblock %.2f, prefetch+precompute %.2f, utxo pass %.2f, "
                    "script wait %.2f, collect %.2f, batch %.2f; parallel UTXO pass in %lld of %d blocks\n",
            useGpu ? "GPU" : "CPU", ms(Chainstate::PH_CHECK), ms(Chainstate::PH_PRECOMPUTE), ms(Chainstate::PH_UTXO),
            ms(Chainstate::PH_SCRIPTS), ms(Chainstate::PH_COLLECT), ms(Chainstate::PH_BATCH),
            (long long)(f.cs->ConnectPhaseMicros(Chainstate::PH_FASTUTXO) - ph0[Chainstate::PH_FASTUTXO]), iters);
    fprintf(stderr, "# %s: parallel UTXO pass (ms/block): setup %.2f, checks %.2f, undo+jobs %.2f, view updates %.2f\n",
            useGpu ? "GPU" : "CPU", ms(Chainstate::PH_FU_SETUP), ms(Chainstate::PH_FU_CHECKS), ms(Chainstate::PH_FU_UNDO),
            ms(Chainstate::PH_FU_APPLY));
    SetGpuSigThreshold(thr);
}
} // namespace

static void ConnectBlock8MB_CPU(State& st) { ConnectBigBlock(st, false, 0); }
static void ConnectBlock8MB_GPU(State& st) {
    if (!gpu::GpuAvailable()) return;
    ConnectBigBlock(st, true, 0);
}
static void ConnectBlock8MB_160kSigops_CPU(State& st) { ConnectBigBlock(st, false, 1); }
static void ConnectBlock8MB_160kSigops_GPU(State& st) {
    if (!gpu::GpuAvailable()) return;
    ConnectBigBlock(st, true, 1);
}
static void ConnectBlock8MB_Multisig_CPU(State& st) { ConnectBigBlock(st, false, 2); }
static void ConnectBlock8MB_Multisig_GPU(State& st) {
    if (!gpu::GpuAvailable()) return;
    ConnectBigBlock(st, true, 2);
}
// Script evaluation of one worst-case P2SH input (<pk> (2DUP CHECKSIGVERIFY) x100 CHECKSIG, the
// 160k-sigop block's redeem script) with every CHECKSIG deferred into a batch sink: the per-input
// CPU cost that block validation pays before the batched ECDSA checks.
static void ScriptP2SH101_Deferred(State& st) {
    CKey key;
    key.MakeNewKey(true);
    const CPubKey pub = key.GetPubKey();
    CScript redeem;
    redeem << std::vector<unsigned char>(pub.begin(), pub.end());
    for (int i = 0; i < 100; i++) redeem << OP_2DUP << OP_CHECKSIGVERIFY;
    redeem << OP_CHECKSIG;
    const CScript spk = GetScriptForDestination(CScriptID(redeem));
    const uint32_t hashType = SIGHASH_ALL | SIGHASH_FORKID;
    CMutableTransaction m;
    m.vin.resize(1);
    m.vin[0].prevout = COutPoint(uint256S("01"), 0);
    m.vout.push_back(CTxOut(1000, spk));
    const Amount amount = 2000;
    {
        const CTransaction u(m);
        std::vector<unsigned char> sig;
        key.Sign(SignatureHash(redeem, u, 0, hashType, amount), sig);
        sig.push_back((unsigned char)hashType);
        m.vin[0].scriptSig = CScript() << sig << std::vector<unsigned char>(redeem.begin(), redeem.end());
    }
    const CTransaction tx(m);
    const PrecomputedTransactionData txdata(tx);
    const uint32_t flags = MANDATORY_SCRIPT_VERIFY_FLAGS | SCRIPT_VERIFY_DERSIG;
    std::vector<DeferredSigCheck> sink;
    while (st.KeepRunning()) {
        sink.clear();
        DeferringSignatureChecker chk(&tx, 0, amount, &txdata, &sink);
        ScriptError err;
        if (!VerifyScript(tx.vin[0].scriptSig, spk, flags, chk, &err) || sink.size() != 101) {
            fprintf(stderr, "ScriptP2SH101_Deferred: %s, %zu checks\n", ScriptErrorString(err), sink.size());
            exit(1);
        }
    }
}
BENCHMARK(ScriptP2SH101_Deferred);

// One P2PKH input through the interpreter with its CHECKSIG deferred (what each of IBD's 40k
// script jobs per block does before the batch): sighash, stack, HASH160; no ECDSA
static void ScriptP2PKH_Deferred(State& st) {
    CKey key;
    key.MakeNewKey(true);
    const CPubKey pub = key.GetPubKey();
    const CScript spk = GetScriptForDestination(pub.GetID());
    const uint32_t hashType = SIGHASH_ALL | SIGHASH_FORKID;
    CMutableTransaction m;
    m.vin.resize(2);
    m.vin[0].prevout = COutPoint(uint256S("01"), 0);
    m.vin[1].prevout = COutPoint(uint256S("02"), 1);
    m.vout.push_back(CTxOut(1000, spk));
    m.vout.push_back(CTxOut(1000, spk));
    const Amount amount = 2000;
    {
        const CTransaction u(m);
        std::vector<unsigned char> sig;
        key.Sign(SignatureHash(spk, u, 0, hashType, amount), sig);
        sig.push_back((unsigned char)hashType);
        m.vin[0].scriptSig = CScript() << sig << std::vector<unsigned char>(pub.begin(), pub.end());
    }
    const CTransaction tx(m);
    const PrecomputedTransactionData txdata(tx);
    const uint32_t flags = MANDATORY_SCRIPT_VERIFY_FLAGS | SCRIPT_VERIFY_DERSIG;
    std::vector<DeferredSigCheck> sink;
    sink.reserve(1 << 16);
    while (st.KeepRunning()) {
        sink.clear();
        for (int r = 0; r < 1000; r++) {
            DeferringSignatureChecker chk(&tx, 0, amount, &txdata, &sink);
            ScriptError err;
            if (!VerifyScript(tx.vin[0].scriptSig, spk, flags, chk, &err)) {
                fprintf(stderr, "ScriptP2PKH_Deferred: %s\n", ScriptErrorString(err));
                exit(1);
            }
        }
    }
}
BENCHMARK(ScriptP2PKH_Deferred);

BENCHMARK(ConnectBlock8MB_CPU);
BENCHMARK(ConnectBlock8MB_GPU);
BENCHMARK(ConnectBlock8MB_160kSigops_CPU);
BENCHMARK(ConnectBlock8MB_160kSigops_GPU);
BENCHMARK(ConnectBlock8MB_Multisig_CPU);
BENCHMARK(ConnectBlock8MB_Multisig_GPU);

// ------------------------------------------------------------------ IBD
// IbdPipeline_Seq_{CPU,GPU}: a fresh node connects -ibdblocks consecutive big blocks (default
// 50; each ~7.3 MB: 20,000 2-in/2-out P2PKH spends of the previous block's outputs, 40,000
// signatures). The blocks arrive last-to-first, so nothing connects until the first one lands
// and then the whole run connects in ActivateBestChain steps, one block at a time (with the GPU:
// each block's UTXO pass in place on the tip, and the next block's read-only pass overlapping
// its signature batch - -connectinplace, -connectlookahead). Reported: ms per block (one
// iteration = the whole run). The round-3..5 "Pipe" variant (-connectpipeline, layered per-block
// views) was removed in round 6: it lost to this path (profiles/connect_r6.md).
namespace {
struct IbdFixture {
    std::vector<std::shared_ptr<const CBlock>> setup, run; // setup: to the fork + fan-out; run: timed
    bool built = false;
};
IbdFixture& Ibd() {
    static IbdFixture f;
    if (f.built) return f;
    f.built = true;
    const int nBlocks = (int)gArgs.GetArg("-ibdblocks", (int64_t)50);
    SelectParams("regtest");
    ChainstateOptions o;
    o.memoryOnly = true;
    char tmpl[] = "/tmp/bench_bcp_ibd_XXXXXX";
    if (!mkdtemp(tmpl)) throw std::runtime_error("bench: mkdtemp failed");
    o.datadir = tmpl;
    o.useGpu = false; // the builder only assembles; validation speed is measured on fresh nodes
    o.scriptThreads = (int)gArgs.GetArg("-par", (int64_t)std::min(16, std::max(2, GetNumCores())));
    o.parallelUtxoMinTx = (size_t)gArgs.GetArg("-parallelutxo", (int64_t)o.parallelUtxoMinTx);
    Chainstate cs(Params(), o);
    CTxMemPool pool;
    std::string err;
    if (!cs.InitBlockIndex(err)) throw std::runtime_error("bench: " + err);
    cs.SetMempool(&pool);
    CBasicKeyStore ks;
    CKey key;
    key.MakeNewKey(true);
    ks.AddKey(key);
    const CScript spk = GetScriptForDestination(key.GetPubKey().GetID());
    const uint32_t hashType = SIGHASH_ALL | SIGHASH_FORKID;
    auto connect = [&](const CBlock& b, std::vector<std::shared_ptr<const CBlock>>& into) {
        auto pb = std::make_shared<const CBlock>(b);
        bool fNew = false;
        CValidationState st;
        if (!cs.ProcessNewBlock(pb, true, &fNew, &st)) throw std::runtime_error("bench: " + FormatStateMessage(st));
        into.push_back(pb);
    };
    std::vector<CTransactionRef> coinbases;
    const int forkHeight = Params().GetConsensus().BCPHeight;
    while (cs.HeightNow() < forkHeight + 1) {
        CBlock b = MakeBlock(cs, pool, spk, {});
        coinbases.push_back(b.vtx[0]);
        connect(b, f.setup);
    }
    const int NFAN = 20, NOUT = 2000, NTX = 20000; // 40,000 outputs carried from block to block
    std::vector<COutPoint> outs;
    std::vector<Amount> vals;
    for (int c0 = 0; c0 < NFAN; c0 += 8) {
        std::vector<CTransactionRef> v;
        for (int c = c0; c < std::min(NFAN, c0 + 8); c++) {
            const CTransaction& cb = *coinbases[c];
            CMutableTransaction m;
            m.vin.resize(1);
            m.vin[0].prevout = COutPoint(cb.GetHash(), 0);
            const Amount each = (cb.vout[0].nValue - 100000) / NOUT;
            for (int k = 0; k < NOUT; k++) m.vout.push_back(CTxOut(each, spk));
            if (!SignSignature(ks, cb.vout[0].scriptPubKey, m, 0, cb.vout[0].nValue, hashType))
                throw std::runtime_error("bench: fan-out signing failed");
            const CTransactionRef t = MakeTransactionRef(std::move(m));
            for (int k = 0; k < NOUT; k++) {
                outs.push_back(COutPoint(t->GetHash(), (uint32_t)k));
                vals.push_back(t->vout[k].nValue);
            }
            v.push_back(t);
        }
        connect(MakeBlock(cs, pool, spk, v), f.setup);
    }
    WorkerPool wp(std::min(16, std::max(2, GetNumCores())));
    for (int b = 0; b < nBlocks; b++) {
        std::vector<CMutableTransaction> txs(NTX);
        std::atomic<bool> fail{false};
        wp.ParallelFor(NTX, [&](size_t t) {
            CMutableTransaction& m = txs[t];
            const Amount in = vals[2 * t] + vals[2 * t + 1];
            for (int k = 0; k < 2; k++) m.vin.emplace_back(CTxIn(outs[2 * t + k]));
            m.vout.push_back(CTxOut(in / 2 - 300, spk));
            m.vout.push_back(CTxOut(in / 2 - 300, spk));
            for (int k = 0; k < 2; k++)
                if (!SignSignature(ks, spk, m, k, vals[2 * t + k], hashType)) fail = true;
        }, 32);
        if (fail) throw std::runtime_error("bench: IBD signing failed");
        std::vector<CTransactionRef> refs;
        refs.reserve(NTX);
        for (int t = 0; t < NTX; t++) {
            refs.push_back(MakeTransactionRef(std::move(txs[t])));
            for (int k = 0; k < 2; k++) {
                outs[2 * t + k] = COutPoint(refs.back()->GetHash(), (uint32_t)k);
                vals[2 * t + k] = refs.back()->vout[k].nValue;
            }
        }
        connect(MakeBlock(cs, pool, spk, refs), f.run);
        if (b % 10 == 9) fprintf(stderr, "# ibd fixture: %d/%d blocks built\n", b + 1, nBlocks);
    }
    fprintf(stderr, "# ibd fixture: %zu setup blocks, %zu big blocks of %zu bytes\n", f.setup.size(), f.run.size(),
            GetSerializeSize(*f.run[0], PROTOCOL_VERSION));
    return f;
}

void IbdRun(State& st, bool useGpu, int pipeline) {
    IbdFixture& f = Ibd();
    const size_t thr = GetGpuSigThreshold();
    SetGpuSigThreshold(useGpu ? DEFAULT_GPU_SIG_THRESHOLD : SIZE_MAX);
    double totalMs = 0;
    int iters = 0;
    while (st.KeepRunning()) {
        ChainstateOptions o;
        o.memoryOnly = true;
        char tmpl[] = "/tmp/bench_bcp_ibdrun_XXXXXX";
        if (!mkdtemp(tmpl)) throw std::runtime_error("bench: mkdtemp failed");
        o.datadir = tmpl;
        o.useGpu = useGpu;
        o.connectInPlace = gArgs.GetBoolArg("-connectinplace", o.connectInPlace);
        o.connectLookahead = gArgs.GetBoolArg("-connectlookahead", o.connectLookahead);
        // -ibdab=inplace|lookahead: alternate that option on (odd runs) and off (even runs), for
        // an interleaved A/B in one process over one fixture
        const std::string ab = gArgs.GetArg("-ibdab", "");
        if (ab == "inplace") o.connectInPlace = iters % 2 == 1;
        if (ab == "lookahead") o.connectLookahead = iters % 2 == 1;
        o.scriptThreads = (int)gArgs.GetArg("-par", (int64_t)std::min(16, std::max(2, GetNumCores())));
        o.parallelUtxoMinTx = (size_t)gArgs.GetArg("-parallelutxo", (int64_t)o.parallelUtxoMinTx);
        Chainstate cs(Params(), o);
        std::string err;
        if (!cs.InitBlockIndex(err)) throw std::runtime_error("bench: " + err);
        auto feed = [&](const std::shared_ptr<const CBlock>& b) {
            bool fNew = false;
            CValidationState vs;
            if (!cs.ProcessNewBlock(b, true, &fNew, &vs)) throw std::runtime_error("bench: " + FormatStateMessage(vs));
        };
        for (const auto& b : f.setup) feed(b);
        // headers first, then the blocks last-to-first: the run connects once the first arrives
        std::vector<CBlockHeader> hdrs;
        for (const auto& b : f.run) hdrs.push_back(b->GetBlockHeader());
        CValidationState hs;
        if (!cs.ProcessNewBlockHeaders(hdrs, hs)) throw std::runtime_error("bench: headers " + FormatStateMessage(hs));
        for (size_t i = f.run.size(); i-- > 1;) feed(f.run[i]);
        int64_t ph0[Chainstate::PH_COUNT];
        for (int k = 0; k < Chainstate::PH_COUNT; k++) ph0[k] = cs.ConnectPhaseMicros((Chainstate::ConnectPhase)k);
        const int64_t t0 = GetTimeMicros();
        feed(f.run[0]);
        const int64_t t1 = GetTimeMicros();
        {
            // where the run's time goes around ConnectTip (ActivateBestChain phases, per block)
            const double nb = (double)f.run.size();
            auto ms = [&](Chainstate::ConnectPhase k) { return 0.001 * (cs.ConnectPhaseMicros(k) - ph0[k]) / nb; };
            const double total = 0.001 * (t1 - t0) / nb;
            const double tip = ms(Chainstate::PH_ABC_TIP);
            fprintf(stderr,
                    "# ibd %s pipeline=%d in_place=%d (ms/block): total %.2f = ConnectTip %.2f + outside %.2f [accept %.2f, find %.3f, "
                    "step-other %.2f, signals %.2f, reap %.2f, notify %.2f, checkindex %.2f, flush %.2f]; "
                    "inside ConnectTip: read %.2f, connectblock %.2f [checkblock %.2f, prefetch %.2f, utxo %.2f, "
                    "scripts %.2f, batch %.2f, undo %.2f], view-flush %.2f, flushstate %.2f, post %.2f; recent-block cache "
                    "hits %llu, misses %llu\n",
                    useGpu ? "GPU" : "CPU", pipeline, (int)o.connectInPlace, total, tip, total - tip, ms(Chainstate::PH_ACCEPT),
                    ms(Chainstate::PH_ABC_FIND), ms(Chainstate::PH_ABC_STEP) - tip, ms(Chainstate::PH_ABC_SIGNALS),
                    ms(Chainstate::PH_ABC_REAP), ms(Chainstate::PH_ABC_NOTIFY), ms(Chainstate::PH_ABC_CHECKINDEX),
                    ms(Chainstate::PH_ABC_FLUSH), ms(Chainstate::PH_TIP_READ), ms(Chainstate::PH_TIP_CONNECT),
                    ms(Chainstate::PH_CHECK), ms(Chainstate::PH_PRECOMPUTE), ms(Chainstate::PH_UTXO),
                    ms(Chainstate::PH_SCRIPTS), ms(Chainstate::PH_BATCH), ms(Chainstate::PH_UNDO), ms(Chainstate::PH_TIP_FLUSH),
                    ms(Chainstate::PH_TIP_WRITE), ms(Chainstate::PH_TIP_POST),
                    (unsigned long long)cs.RecentBlockHits(), (unsigned long long)cs.RecentBlockMisses());
            fprintf(stderr, "# ibd fast-utxo sub-phases (ms/block): setup %.2f checks %.2f undo %.2f apply %.2f; "
                    "lookahead wait %.2f, adopted by %lld of %zu blocks\n",
                    ms(Chainstate::PH_FU_SETUP), ms(Chainstate::PH_FU_CHECKS), ms(Chainstate::PH_FU_UNDO),
                    ms(Chainstate::PH_FU_APPLY), ms(Chainstate::PH_LA_WAIT),
                    (long long)(cs.ConnectPhaseMicros(Chainstate::PH_LA_USED) - ph0[Chainstate::PH_LA_USED]), f.run.size());
        }
        if (cs.HeightNow() != f.run.size() + f.setup.size()) {
            fprintf(stderr, "IBD run ended at height %d\n", cs.HeightNow());
            exit(1);
        }
        {
            // the undo records written during the run read back with matching checksums
            std::lock_guard<CCriticalSection> l(cs.cs());
            for (const CBlockIndex* p = cs.Tip(); p && p->nHeight > (int)f.setup.size(); p = p->pprev) {
                CBlockUndo u;
                if (!UndoReadFromDisk(u, p->GetUndoPos(), p->pprev->GetBlockHash()) || u.vtxundo.size() < 20000) {
                    fprintf(stderr, "IBD run: undo record of height %d unreadable\n", p->nHeight);
                    exit(1);
                }
            }
        }
        totalMs += (t1 - t0) / 1000.0;
        iters++;
        printf("{\"bench\": \"IbdPipelineRun\", \"gpu\": %s, \"pipeline\": %d, \"in_place\": %s, \"lookahead\": %s, \"iter\": %d, \"ms_per_block\": %.2f}\n",
               useGpu ? "true" : "false", pipeline, o.connectInPlace ? "true" : "false", o.connectLookahead ? "true" : "false", iters, (t1 - t0) / 1000.0 / f.run.size());
        fflush(stdout);
        const std::string cmd = std::string("rm -rf '") + tmpl + "'";
        if (system(cmd.c_str()) != 0) {}
    }
    printf("{\"bench\": \"IbdPipeline\", \"gpu\": %s, \"pipeline\": %d, \"blocks\": %zu, \"ms_per_block\": %.2f}\n",
           useGpu ? "true" : "false", pipeline, f.run.size(), totalMs / iters / f.run.size());
    fflush(stdout);
    SetGpuSigThreshold(thr);
}
} // namespace
static void IbdPipeline_Seq_CPU(State& st) { IbdRun(st, false, 1); }
static void IbdPipeline_Seq_GPU(State& st) {
    if (gpu::GpuAvailable()) IbdRun(st, true, 1);
}
BENCHMARK(IbdPipeline_Seq_CPU);
BENCHMARK(IbdPipeline_Seq_GPU);

int main(int argc, char* argv[]) {
    gArgs.ParseParameters(argc, argv);
    if (gArgs.IsArgSet("-?") || gArgs.IsArgSet("-h") || gArgs.IsArgSet("-help")) {
        printf("Usage: bench_bcp [-filter=<regex>] [-time=<seconds per bench>] [-list] [-datadir=bench/data]\n"
               "                 [-par=<script threads>] [-ibdblocks=<n>] [-kvcoins=<n>] [-kvdbcache=<MiB>]\n"
               "                 [-parallelutxo=<min txs>] [-ecdsaminshard=<signatures>] [-debug=<category>]\n"
               "                 [-shardplan] (print the GPU verify shard plans for 1, 2 and 8 devices)\n"
               "                 [-connectinplace=0|1] [-connectlookahead=0|1] [-ibdab=inplace|lookahead]\n"
               "                 (IBD: alternate one of those options run by run) [-tipcoins=<n>]\n");
        return 0;
    }
    { // default: <dir of the binary>/../bench/data, so the working directory does not matter
        char exe[4096];
        const ssize_t len = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
        if (len > 0) {
            std::string p(exe, (size_t)len);
            p = p.substr(0, p.find_last_of('/'));
            g_dataDir = p + "/../bench/data";
        }
    }
    g_dataDir = gArgs.GetArg("-datadir", g_dataDir);
    if (gArgs.IsArgSet("-debug")) { // e.g. -debug=bench: ConnectBlock's phase timers on stderr-side console
        LogInit("", true, false);
        LogEnableCategory(gArgs.GetArg("-debug", "bench"));
    }
    if (gArgs.IsArgSet("-shardplan")) { // the verify service's shard plans for 1, 2 and 8 devices
        for (int ndev : {1, 2, 8}) {
            std::vector<int> lanes; // the default lane list: every device, twice, round-robin
            for (int rep = 0; rep < 2; rep++)
                for (int d = 0; d < ndev; d++) lanes.push_back(d);
            for (size_t n : {(size_t)512, (size_t)42000, (size_t)199000}) {
                const auto plan = PlanShards(n, lanes, 4096, 65536); // the ECDSA defaults
                printf("ecdsa devices=%d n=%zu shards=%zu:", ndev, n, plan.size());
                for (const auto& sh : plan) printf(" [lane %zu dev %d: %zu]", sh.lane, lanes[sh.lane], sh.hi - sh.lo);
                printf("\n");
            }
            for (size_t n : {(size_t)160, (size_t)2000}) {
                const auto plan = PlanShards(n, lanes, 256, 2048); // the header defaults
                printf("headers devices=%d n=%zu shards=%zu:", ndev, n, plan.size());
                for (const auto& sh : plan) printf(" [dev %d: %zu]", lanes[sh.lane], sh.hi - sh.lo);
                printf("\n");
            }
        }
        return 0;
    }
    const std::regex filter(gArgs.GetArg("-filter", ".*"));
    const double minTime = atof(gArgs.GetArg("-time", "1.0").c_str());
    if (gArgs.IsArgSet("-list")) {
        for (const auto& b : bench::Registry()) printf("%s\n", b.first.c_str());
        return 0;
    }
    printf("# %-32s %10s %14s %14s %14s %14s %14s %14s\n", "Benchmark", "iterations", "total", "min", "max", "median",
           "p25", "p75");
    for (const auto& b : bench::Registry()) {
        if (!std::regex_match(b.first, filter)) continue;
        State st(b.first, minTime);
        b.second(st);
        st.Report();
    }
    return 0;
}
