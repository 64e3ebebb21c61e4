// kvstore_tests: the log-structured KV store behind the chainstate, block index and wallet.
// Parity: reference src/test/dbwrapper_tests.cpp (read/write, batches, iterators, existing-data
// reopen) for the CDBWrapper contract, plus what LevelDB guarantees there implicitly: atomic
// batches across crashes, torn-log recovery, and bounded memory under a growing key set.
#include "test/unittest.h"

#include "node/kvstore.h"
#include "util/strencodings.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <thread>
#include <unistd.h>

using namespace bcp;

namespace {

std::string TempDir(const char* tag) {
    char buf[] = "/tmp/bcp_kvtest_XXXXXX";
    const char* d = mkdtemp(buf);
    REQUIRE(d != nullptr);
    return std::string(d) + "/" + tag;
}
void RmRf(const std::string& dir) {
    const std::string cmd = "rm -rf '" + dir.substr(0, dir.rfind('/')) + "'";
    if (std::system(cmd.c_str()) != 0) {}
}

KVOptions Small() {
    KVOptions o;
    o.memtableBytes = 16 << 10; // many flushes
    o.blockCacheBytes = 64 << 10;
    o.blockBytes = 512;
    o.maxSegments = 4; // frequent merges
    o.mergeWidth = 3;
    return o;
}

std::string K(uint64_t i) { return strprintf("k%08llu", (unsigned long long)i); }

// The store's full contents equal the model, both by iteration and by point reads.
bool SameAsModel(const KVStore& db, const std::map<std::string, std::string>& model, const char* where) {
    auto it = db.NewIterator();
    auto m = model.begin();
    size_t n = 0;
    for (it->SeekToFirst(); it->Valid(); it->Next(), ++m, ++n) {
        std::string v;
        if (m == model.end() || it->RawKey() != m->first || !it->RawValue(v) || v != m->second) {
            test::RecordFailure(strprintf("%s: iteration differs at #%zu (%s)", where, n, it->RawKey().c_str()), __FILE__,
                                __LINE__);
            return false;
        }
    }
    if (m != model.end()) {
        test::RecordFailure(strprintf("%s: iteration ended early at #%zu", where, n), __FILE__, __LINE__);
        return false;
    }
    for (const auto& kv : model) {
        std::string v;
        if (!db.ReadRaw(kv.first, v) || v != kv.second) {
            test::RecordFailure(strprintf("%s: point read of %s", where, kv.first.c_str()), __FILE__, __LINE__);
            return false;
        }
    }
    return true;
}

} // namespace

TEST_CASE(kvstore_tests, model_random_ops_with_flushes_merges_reopens) {
    FastRandomContext rng(true);
    const std::string dir = TempDir("db");
    std::map<std::string, std::string> model;
    {
        std::unique_ptr<KVStore> db(new KVStore(dir, false, true, Small()));
        for (int round = 0; round < 30; round++) {
            KVBatch b;
            const int nops = 1 + rng.randrange(200);
            for (int i = 0; i < nops; i++) {
                const std::string k = K(rng.randrange(3000));
                if (rng.randrange(4) == 0) {
                    b.EraseRaw(k);
                    model.erase(k);
                } else {
                    const std::string v = strprintf("v%d-%d-", round, i) + std::string(rng.randrange(60), 'x');
                    b.WriteRaw(k, v);
                    model[k] = v;
                }
            }
            REQUIRE(db->WriteBatch(b, rng.randrange(4) == 0));
            // absent keys read as absent, also past every segment's range
            std::string v;
            CHECK(!db->ReadRaw("a-before-everything", v));
            CHECK(!db->ReadRaw("zzz-after-everything", v));
            if (round % 7 == 6) {
                db.reset(); // one instance per directory
                db.reset(new KVStore(dir, false, false, Small())); // reopen: logs replayed
                CHECK_THROWS(KVStore(dir, false, false, Small()));
            }
            if (round % 5 == 4 && !SameAsModel(*db, model, "round")) return;
        }
        const KVStats st = db->Stats();
        CHECK(st.flushes > 0 || st.segments > 0);
        CHECK(st.segments <= 8u);
        // seek lands on the first key >= target, tombstones skipped
        auto it = db->NewIterator();
        for (int t = 0; t < 50; t++) {
            const std::string target = K(rng.randrange(3100));
            it->Seek(target);
            auto m = model.lower_bound(target);
            CHECK_EQ(it->Valid(), m != model.end());
            if (it->Valid() && m != model.end()) CHECK_EQ(it->RawKey(), m->first);
        }
        db->Compact();
        CHECK_EQ(db->Stats().segments, 1u);
        SameAsModel(*db, model, "after compact");
        CHECK_EQ(db->Count(), model.size());
        CHECK_EQ(db->IsEmpty(), model.empty());
    }
    {
        KVStore db(dir, false, false, Small());
        SameAsModel(db, model, "final reopen");
        // erase everything: empty after a full compaction, and after reopening
        KVBatch b;
        for (const auto& kv : model) b.EraseRaw(kv.first);
        REQUIRE(db.WriteBatch(b, true));
        db.Compact();
        CHECK(db.IsEmpty());
        CHECK_EQ(db.Stats().segments, 0u);
    }
    {
        KVStore db(dir, false, false, Small());
        CHECK(db.IsEmpty());
    }
    RmRf(dir);
}

TEST_CASE(kvstore_tests, memory_only_matches_disk) {
    FastRandomContext rng(true);
    KVStore mem("", true);
    const std::string dir = TempDir("db");
    KVStore disk(dir, false, true, Small());
    std::map<std::string, std::string> model;
    for (int i = 0; i < 4000; i++) {
        KVBatch a, b;
        const std::string k = K(rng.randrange(500));
        if (rng.randrange(3) == 0) {
            a.EraseRaw(k);
            b.EraseRaw(k);
            model.erase(k);
        } else {
            const std::string v = std::to_string(i);
            a.WriteRaw(k, v);
            b.WriteRaw(k, v);
            model[k] = v;
        }
        REQUIRE(mem.WriteBatch(a));
        REQUIRE(disk.WriteBatch(b));
    }
    SameAsModel(mem, model, "memory");
    SameAsModel(disk, model, "disk");
    CHECK_EQ(mem.EstimateSize("k", "l") > 0, !model.empty());
    RmRf(dir);
}

TEST_CASE(kvstore_tests, torn_log_tail_keeps_a_batch_prefix) {
    // Each batch i sets ctr = i and writes 20 keys b<i>-<j>; truncating the log anywhere must
    // leave exactly batches 0..c (no partial batch), whatever segments hold.
    FastRandomContext rng(true);
    for (int trial = 0; trial < 12; trial++) {
        const std::string dir = TempDir("db");
        const int batches = 40 + rng.randrange(60);
        {
            KVOptions o = Small();
            o.memtableBytes = 1 << 20; // everything stays in the log
            KVStore db(dir, false, true, o);
            for (int i = 0; i < batches; i++) {
                KVBatch b;
                b.WriteRaw("ctr", std::to_string(i));
                for (int j = 0; j < 20; j++) b.WriteRaw(strprintf("b%04d-%02d", i, j), std::string(30, 'a' + j));
                REQUIRE(db.WriteBatch(b));
            }
        }
        // find the log and tear it at a random byte
        std::string log;
        for (int n = 1; n < 10 && log.empty(); n++) {
            const std::string p = strprintf("%s/kv-%06d.log", dir.c_str(), n);
            struct stat st;
            if (stat(p.c_str(), &st) == 0 && st.st_size > 0) log = p;
        }
        REQUIRE(!log.empty());
        struct stat st;
        REQUIRE(stat(log.c_str(), &st) == 0);
        const off_t cut = (off_t)rng.randrange((uint64_t)st.st_size);
        REQUIRE(truncate(log.c_str(), cut) == 0);
        KVStore db(dir, false, false, Small());
        std::string ctr;
        int c = -1;
        if (db.ReadRaw("ctr", ctr)) c = atoi(ctr.c_str());
        CHECK(c < batches);
        size_t keys = 0;
        auto it = db.NewIterator();
        for (it->SeekToFirst(); it->Valid(); it->Next()) {
            if (it->RawKey() == "ctr") continue;
            ++keys;
            CHECK(atoi(it->RawKey().c_str() + 1) <= c);
        }
        CHECK_EQ(keys, (size_t)(c + 1) * 20);
        // the store keeps working after recovery
        KVBatch b;
        b.WriteRaw("after", "1");
        CHECK(db.WriteBatch(b, true));
        RmRf(dir);
    }
}

TEST_CASE(kvstore_tests, crash_mid_batch_stream) {
    // A child process writes batches (with flushes and merges running underneath) and is
    // SIGKILLed at a random moment; the reopened store must hold a complete prefix of batches.
    FastRandomContext rng(true);
    const std::string dir = TempDir("db");
    int total = 0;
    for (int trial = 0; trial < 6; trial++) {
        const pid_t pid = fork();
        REQUIRE(pid >= 0);
        if (pid == 0) {
            KVStore db(dir, false, false, Small());
            std::string ctr;
            int i = db.ReadRaw("ctr", ctr) ? atoi(ctr.c_str()) + 1 : 0;
            for (;; i++) {
                KVBatch b;
                b.WriteRaw("ctr", std::to_string(i));
                for (int j = 0; j < 8; j++) b.WriteRaw(strprintf("c%07d-%d", i, j), std::string(40, 'q'));
                if (i >= 8) // a sliding window: delete an older batch's keys in the same batch
                    for (int j = 0; j < 8; j++) b.EraseRaw(strprintf("c%07d-%d", i - 8, j));
                if (!db.WriteBatch(b)) _exit(3);
            }
        }
        usleep(20000 + (useconds_t)rng.randrange(150000));
        kill(pid, SIGKILL);
        int status = 0;
        waitpid(pid, &status, 0);
        CHECK(WIFSIGNALED(status));
        KVStore db(dir, false, false, Small());
        std::string ctr;
        REQUIRE(db.ReadRaw("ctr", ctr));
        const int c = atoi(ctr.c_str());
        CHECK(c >= total - 1);
        total = c + 1;
        // exactly the keys of batches max(0, c-7) .. c
        std::map<std::string, std::string> model;
        for (int i = std::max(0, c - 7); i <= c; i++)
            for (int j = 0; j < 8; j++) model[strprintf("c%07d-%d", i, j)] = std::string(40, 'q');
        model["ctr"] = ctr;
        if (!SameAsModel(db, model, "after crash")) break;
    }
    CHECK(total > 100);
    RmRf(dir);
}

TEST_CASE(kvstore_tests, concurrent_readers_during_merges) {
    const std::string dir = TempDir("db");
    KVStore db(dir, false, true, Small());
    // a fixed key set that never changes, plus churn in another key range
    {
        KVBatch b;
        for (int i = 0; i < 2000; i++) b.WriteRaw(strprintf("fixed%05d", i), std::to_string(i));
        REQUIRE(db.WriteBatch(b));
    }
    std::atomic<bool> stop{false};
    std::atomic<int> errors{0};
    std::thread reader([&] {
        FastRandomContext r(true);
        while (!stop) {
            const int i = (int)r.randrange(2000);
            std::string v;
            if (!db.ReadRaw(strprintf("fixed%05d", i), v) || v != std::to_string(i)) errors++;
            auto it = db.NewIterator();
            it->Seek(std::string("fixed"));
            int n = 0;
            for (; it->Valid() && it->RawKey().compare(0, 5, "fixed") == 0; it->Next()) n++;
            if (n != 2000) errors++;
        }
    });
    for (int round = 0; round < 300; round++) {
        KVBatch b;
        for (int j = 0; j < 40; j++) b.WriteRaw(strprintf("churn%03d-%02d", round % 50, j), std::string(100, 'z'));
        REQUIRE(db.WriteBatch(b));
    }
    stop = true;
    reader.join();
    CHECK_EQ(errors.load(), 0);
    CHECK(db.Stats().merges > 0);
    RmRf(dir);
}

TEST_CASE(kvstore_tests, legacy_log_is_migrated) {
    // A pre-segment store: one kv.log of v1 records (magic, len, crc32c, ops). Build one by
    // hand, open it, and find the data in a segment with the old log gone.
    const std::string dir = TempDir("db");
    REQUIRE(system(("mkdir -p '" + dir + "'").c_str()) == 0);
    auto crc32c = [](const std::string& s) {
        uint32_t c = 0xFFFFFFFFu;
        for (unsigned char ch : s) {
            c ^= ch;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (0x82F63B78u ^ (c >> 1)) : (c >> 1);
        }
        return c ^ 0xFFFFFFFFu;
    };
    auto rec = [&](const std::string& payload) {
        std::string r;
        const uint32_t magic = 0xB7C0DB01, len = (uint32_t)payload.size(), crc = crc32c(payload);
        r.append((const char*)&magic, 4);
        r.append((const char*)&len, 4);
        r.append((const char*)&crc, 4);
        return r + payload;
    };
    auto put = [](const std::string& k, const std::string& v) {
        return std::string(1, '\x01') + (char)k.size() + k + (char)v.size() + v;
    };
    auto del = [](const std::string& k) { return std::string(1, '\x02') + (char)k.size() + k; };
    const std::string log = rec(put("alpha", "1") + put("beta", "2")) + rec(del("alpha") + put("gamma", "3"));
    FILE* f = fopen((dir + "/kv.log").c_str(), "wb");
    REQUIRE(f != nullptr);
    fwrite(log.data(), 1, log.size(), f);
    fclose(f);
    {
        KVStore db(dir, false, false, Small());
        std::string v;
        CHECK(!db.ReadRaw("alpha", v));
        CHECK(db.ReadRaw("beta", v) && v == "2");
        CHECK(db.ReadRaw("gamma", v) && v == "3");
        CHECK_EQ(db.Stats().segments, 1u);
        struct stat st;
        CHECK(stat((dir + "/kv.log").c_str(), &st) != 0);
    }
    KVStore db(dir, false, false, Small());
    std::string v;
    CHECK(db.ReadRaw("gamma", v) && v == "3");
    CHECK_EQ(db.Count(), 2u);
    RmRf(dir);
}

TEST_CASE(kvstore_tests, salvage_skips_damage) {
    const std::string dir = TempDir("db");
    std::map<std::string, std::string> model;
    {
        KVStore db(dir, false, true, Small());
        for (int i = 0; i < 600; i++) {
            KVBatch b;
            b.WriteRaw(K(i), std::string(50, 'a' + i % 26));
            model[K(i)] = std::string(50, 'a' + i % 26);
            REQUIRE(db.WriteBatch(b));
        }
        db.Flush();
    }
    uint64_t skipped = 1;
    std::map<std::string, std::string> got = KVStore::Salvage(dir, &skipped);
    CHECK_EQ(skipped, 0u);
    CHECK(got == model);
    // damage a byte in the middle of the first segment: only that block's keys are lost
    std::string seg;
    for (int n = 1; n < 400 && seg.empty(); n++) {
        const std::string p = strprintf("%s/seg-%06d.sst", dir.c_str(), n);
        struct stat st;
        if (stat(p.c_str(), &st) == 0 && st.st_size > 2048) seg = p;
    }
    REQUIRE(!seg.empty());
    FILE* f = fopen(seg.c_str(), "r+b");
    REQUIRE(f != nullptr);
    fseek(f, 100, SEEK_SET);
    fputc(0xEE, f);
    fclose(f);
    got = KVStore::Salvage(dir, &skipped);
    CHECK(skipped > 0);
    CHECK(got.size() < model.size());
    CHECK(got.size() > model.size() / 2);
    for (const auto& kv : got) CHECK(model.count(kv.first) && model[kv.first] == kv.second);
    RmRf(dir);
}

// A damaged segment block is an error, never a missing key (reference dbwrapper_error): the
// chainstate would otherwise read disk damage as a spent coin and reject a valid block.
TEST_CASE(kvstore_tests, corrupt_block_reads_as_an_error) {
    const std::string dir = TempDir("db");
    std::map<std::string, std::string> model;
    {
        KVStore db(dir, false, true, Small());
        for (int i = 0; i < 600; i++) {
            KVBatch b;
            b.WriteRaw(K(i), std::string(50, 'a' + i % 26));
            model[K(i)] = std::string(50, 'a' + i % 26);
            REQUIRE(db.WriteBatch(b));
        }
        db.Flush();
    }
    std::string seg;
    for (int n = 1; n < 400 && seg.empty(); n++) {
        const std::string p = strprintf("%s/seg-%06d.sst", dir.c_str(), n);
        struct stat st;
        if (stat(p.c_str(), &st) == 0 && st.st_size > 2048) seg = p;
    }
    REQUIRE(!seg.empty());
    FILE* f = fopen(seg.c_str(), "r+b");
    REQUIRE(f != nullptr);
    fseek(f, 100, SEEK_SET);
    fputc(0xEE, f);
    fclose(f);
    KVStore db(dir, false, false, Small());
    size_t thrown = 0, ok = 0;
    for (const auto& kv : model) {
        std::string v;
        try {
            const bool found = db.ReadRaw(kv.first, v);
            CHECK(found); // never "absent"
            CHECK(v == kv.second);
            ++ok;
        } catch (const KVCorruption&) {
            ++thrown;
        }
    }
    CHECK(thrown > 0);
    CHECK(ok > model.size() / 2);
    // the batched lookup (CCoinsViewDB::PeekCoins) reports the damage the same way
    std::vector<std::string> keys, vals(model.size());
    for (const auto& kv : model) keys.push_back(kv.first);
    std::vector<uint8_t> found(keys.size());
    bool threw = false;
    try {
        db.ReadRawMany(keys.data(), keys.size(), vals.data(), found.data());
    } catch (const KVCorruption&) {
        threw = true;
    }
    CHECK(threw);
    RmRf(dir);
}

// A failed manifest write (flush or merge) keeps every committed key: the logs the old manifest
// still names are not unlinked, merge inputs are not dropped, and a reopen replays them.
TEST_CASE(kvstore_tests, failed_manifest_write_loses_nothing) {
    for (int mode = 0; mode < 2; mode++) { // 0: during a flush, 1: during a merge (Compact)
        const std::string dir = TempDir("db");
        std::map<std::string, std::string> model;
        {
            KVStore db(dir, false, true, Small());
            for (int i = 0; i < 400; i++) {
                KVBatch b;
                b.WriteRaw(K(i), strprintf("v%d-%d", i, mode));
                REQUIRE(db.WriteBatch(b));
                model[K(i)] = strprintf("v%d-%d", i, mode);
            }
            db.Flush();
            db.InjectFault(KVStore::FAULT_MANIFEST);
            if (mode == 0) {
                for (int i = 400; i < 2000; i++) { // until the background flush fails
                    KVBatch b;
                    b.WriteRaw(K(i), std::string(40, 'x'));
                    if (!db.WriteBatch(b)) break;
                    model[K(i)] = std::string(40, 'x');
                }
            } else {
                db.Compact();
            }
            CHECK(SameAsModel(db, model, mode ? "after failed merge" : "after failed flush"));
        }
        KVStore db(dir, false, false, Small());
        CHECK(SameAsModel(db, model, mode ? "reopened after failed merge" : "reopened after failed flush"));
        RmRf(dir);
    }
}

// A failed segment write keeps the sealed memtable readable and its logs for the replay.
TEST_CASE(kvstore_tests, failed_segment_write_loses_nothing) {
    const std::string dir = TempDir("db");
    std::map<std::string, std::string> model;
    bool refused = false;
    {
        KVStore db(dir, false, true, Small());
        db.InjectFault(KVStore::FAULT_SEGMENT);
        for (int i = 0; i < 3000; i++) {
            KVBatch b;
            b.WriteRaw(K(i), std::string(40, 'a' + i % 26));
            if (!db.WriteBatch(b)) {
                refused = true;
                break;
            }
            model[K(i)] = std::string(40, 'a' + i % 26);
        }
        CHECK(SameAsModel(db, model, "after failed segment write"));
    }
    CHECK(refused); // the store stops taking writes once a flush failed
    KVStore db(dir, false, false, Small());
    CHECK(SameAsModel(db, model, "reopened after failed segment write"));
    RmRf(dir);
}
