// Wallet coin selection and address-book records.
// Parity: reference src/wallet/test/wallet_tests.cpp (coin_selection_tests,
// ApproximateBestSubset) and src/wallet/test/walletdb_tests.cpp (write/erase of name, purpose
// and destdata, which the reference reads back through a fresh CWalletDB). Coins here are
// in-memory wallet transactions; "from me" coins really spend one of the wallet's own outputs.
#include "test/unittest.h"
#include "node/kvstore.h"
#include "wallet/bdbimport.h"
#include "wallet/wallet.h"

#include <cmath>
#include <fstream>
#include <set>
#include <sstream>
#include <deque>
#include <unistd.h>

namespace bcp {
namespace {

typedef std::set<std::pair<const CWalletTx*, unsigned int>> CoinSet;

struct Pool {
    CWallet wallet{"test", "", true};
    std::deque<CWalletTx> txs; // stable addresses for COutput::tx
    std::vector<COutput> coins;
    CKey key;
    uint256 fundingTx; // a wallet-owned output the "from me" coins spend
    uint32_t lockTime = 0;
    Pool() {
        key.MakeNewKey(true);
        wallet.AddKeyPubKey(key, key.GetPubKey());
        CMutableTransaction f;
        f.vin.resize(1);
        f.vout.push_back(CTxOut(COIN, GetScriptForDestination(key.GetPubKey().GetID())));
        CWalletTx wtx(&wallet, MakeTransactionRef(std::move(f)));
        fundingTx = wtx.GetHash();
        WalletLock l(wallet);
        wallet.mapWallet[fundingTx] = wtx;
    }
    // a coin of value v, `depth` confirmations, optionally spending our own output
    void Add(Amount v, int depth = 144, bool fromMe = false) {
        CMutableTransaction t;
        t.nLockTime = lockTime++; // distinct hashes
        if (fromMe) t.vin.push_back(CTxIn(COutPoint(fundingTx, 0)));
        t.vout.push_back(CTxOut(v, CScript() << OP_TRUE));
        txs.emplace_back(&wallet, MakeTransactionRef(std::move(t)));
        coins.push_back({&txs.back(), 0, depth, true, true});
    }
    void Clear() {
        coins.clear();
        txs.clear();
    }
    bool Select(Amount target, int confMine, int confTheirs, CoinSet& set, Amount& value) {
        return wallet.SelectCoinsMinConf(target, confMine, confTheirs, 0, coins, set, value);
    }
};

} // namespace

TEST_CASE(wallet_tests, selection_depths_and_origin) {
    Pool p;
    CoinSet set;
    Amount v = 0;
    CHECK(!p.Select(CENT, 1, 6, set, v)); // nothing at all
    p.Add(2 * CENT, 3);                   // young coin from someone else
    CHECK(!p.Select(2 * CENT, 1, 6, set, v));
    CHECK(p.Select(2 * CENT, 1, 3, set, v));
    CHECK_EQ(v, 2 * CENT);
    p.Add(3 * CENT, 2, true); // young change of our own
    CHECK(p.Select(3 * CENT, 1, 6, set, v)); // our own coins need one confirmation only
    CHECK_EQ(v, 3 * CENT);
    CHECK(!p.Select(3 * CENT, 6, 6, set, v));
    p.Add(40 * CENT); // mature
    CHECK(p.Select(45 * CENT, 1, 3, set, v));
    CHECK_EQ(v, 45 * CENT);
    CHECK(!p.Select(45 * CENT, 1, 6, set, v)); // the 2-cent coin is too young for 6
    CHECK(p.Select(43 * CENT, 1, 6, set, v));
    CHECK_EQ(v, 43 * CENT);
    CHECK(!p.Select(46 * CENT, 1, 1, set, v)); // more than everything
}

TEST_CASE(wallet_tests, selection_subsets_versus_larger_coin) {
    for (int rep = 0; rep < 50; rep++) { // the search is randomised: repeat it
        Pool p;
        CoinSet set;
        Amount v = 0;
        for (int c : {3, 4, 9, 25, 50}) p.Add(c * CENT);
        // an exact single coin wins
        CHECK(p.Select(9 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 9 * CENT);
        CHECK_EQ(set.size(), (size_t)1);
        // an exact subset of the small coins: 3 + 4
        CHECK(p.Select(7 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 7 * CENT);
        CHECK_EQ(set.size(), (size_t)2);
        // 20: the small coins (3+4+9 = 16) cannot reach it, so the smallest larger coin
        CHECK(p.Select(20 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 25 * CENT);
        CHECK_EQ(set.size(), (size_t)1);
        // 15: 3+4+9 = 16 beats the next larger coin (25)
        CHECK(p.Select(15 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 16 * CENT);
        CHECK_EQ(set.size(), (size_t)3);
        p.Add(16 * CENT);
        // now a single 16 ties with 3+4+9: the single larger coin wins a tie
        CHECK(p.Select(15 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 16 * CENT);
        CHECK_EQ(set.size(), (size_t)1);
        // everything, and not a satoshi more
        CHECK(p.Select(107 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 107 * CENT);
        CHECK(!p.Select(107 * CENT + 1, 1, 1, set, v));
        // among larger coins the smallest is used
        for (int c : {2, 3, 5}) p.Add(c * COIN);
        CHECK(p.Select(180 * CENT, 1, 1, set, v));
        CHECK_EQ(v, 2 * COIN);
        CHECK_EQ(set.size(), (size_t)1);
    }
}

TEST_CASE(wallet_tests, selection_avoids_small_change) {
    for (int rep = 0; rep < 50; rep++) {
        Pool p;
        CoinSet set;
        Amount v = 0;
        // only tiny coins: change below MIN_CHANGE is unavoidable, so the target exactly
        for (int i = 1; i <= 6; i++) p.Add(i * MIN_CHANGE / 10);
        CHECK(p.Select(MIN_CHANGE, 1, 1, set, v));
        CHECK_EQ(v, MIN_CHANGE);
        // with a big coin around, the exact subset is still preferred over big change
        p.Add(500 * MIN_CHANGE);
        CHECK(p.Select(MIN_CHANGE, 1, 1, set, v));
        CHECK_EQ(v, MIN_CHANGE);
        p.Clear();
        // small coins that cannot reach target + MIN_CHANGE and have no exact subset: the big coin
        for (int i : {5, 6, 7}) p.Add(i * MIN_CHANGE / 10);
        p.Add(800 * MIN_CHANGE);
        CHECK(p.Select(MIN_CHANGE, 1, 1, set, v));
        CHECK_EQ(v, 800 * MIN_CHANGE);
        CHECK_EQ(set.size(), (size_t)1);
        p.Clear();
        // 0.03 + 1 + 100 for 100.01: all three (change 1.02 is fine); for 99.9: 100 + 1
        p.Add(3 * MIN_CHANGE / 100);
        p.Add(MIN_CHANGE);
        p.Add(100 * MIN_CHANGE);
        CHECK(p.Select(10001 * MIN_CHANGE / 100, 1, 1, set, v));
        CHECK_EQ(v, 10103 * MIN_CHANGE / 100);
        CHECK_EQ(set.size(), (size_t)3);
        CHECK(p.Select(9990 * MIN_CHANGE / 100, 1, 1, set, v));
        CHECK_EQ(v, 101 * MIN_CHANGE);
        CHECK_EQ(set.size(), (size_t)2);
    }
}

TEST_CASE(wallet_tests, selection_many_equal_coins) {
    Pool p;
    CoinSet set, set2;
    Amount v = 0;
    // consolidating 30 equal coins into an amount of 12 of them: exactly 12
    for (int i = 0; i < 30; i++) p.Add(40000 * COIN);
    CHECK(p.Select(480000 * COIN, 1, 1, set, v));
    CHECK_EQ(v, 480000 * COIN);
    CHECK_EQ(set.size(), (size_t)12);
    // hundreds of small inputs: as few as cover target + MIN_CHANGE, or one if a coin suffices
    for (Amount a = 2500; a < COIN; a *= 10) {
        p.Clear();
        for (int i = 0; i < 600; i++) p.Add(a);
        CHECK(p.Select(3000, 1, 1, set, v));
        if (a - 3000 < MIN_CHANGE) {
            const size_t n = (size_t)std::ceil((3000.0 + MIN_CHANGE) / a);
            CHECK_EQ(set.size(), n);
            CHECK_EQ(v, (Amount)n * a);
        } else {
            CHECK_EQ(set.size(), (size_t)1);
            CHECK_EQ(v, a);
        }
    }
    // the choice among identical coins is random
    p.Clear();
    for (int i = 0; i < 100; i++) p.Add(COIN);
    CHECK(p.Select(50 * COIN, 1, 6, set, v));
    CHECK(p.Select(50 * COIN, 1, 6, set2, v));
    CHECK(set != set2);
    int same = 0;
    for (int i = 0; i < 6; i++) {
        CHECK(p.Select(COIN, 1, 6, set, v));
        CHECK(p.Select(COIN, 1, 6, set2, v));
        same += set == set2;
    }
    CHECK(same < 6);
    // sort order of the subset search: many big coins and one small one
    p.Clear();
    for (int i = 0; i < 800; i++) p.Add(1000 * COIN);
    p.Add(3 * COIN);
    CHECK(p.Select(1003 * COIN, 1, 6, set, v));
    CHECK_EQ(v, 1003 * COIN);
    CHECK_EQ(set.size(), (size_t)2);
}

TEST_CASE(walletdb_tests, address_book_records_persist) {
    char tmpl[] = "/tmp/bcp_walletdb_XXXXXX";
    REQUIRE(mkdtemp(tmpl) != nullptr);
    const std::string path = std::string(tmpl) + "/wallet.dat";
    CKey k;
    k.MakeNewKey(true);
    const CTxDestination a = k.GetPubKey().GetID();
    CKey k2;
    k2.MakeNewKey(true);
    const CTxDestination b = k2.GetPubKey().GetID();
    {
        CWallet w("w", path, false);
        std::string err;
        bool first = false;
        REQUIRE(w.Load(err, first));
        CHECK(w.SetAddressBook(a, "alice", "receive"));
        CHECK(w.SetAddressBook(b, "bob", "send"));
        CHECK(w.AddDestData(a, "rr0", "request-0"));
        CHECK(w.AddDestData(a, "used", "1"));
        CHECK(w.AddDestData(b, "rr1", "request-1"));
        CHECK(!w.AddDestData(CTxDestination(), "x", "y")); // no destination, no record
        CHECK(w.EraseDestData(a, "used"));
        CHECK(!w.EraseDestData(a, "never-set"));
        CHECK(w.DelAddressBook(b)); // takes its destdata with it
    }
    {
        CWallet w("w", path, false);
        std::string err;
        bool first = true;
        REQUIRE(w.Load(err, first));
        CHECK(!first);
        REQUIRE(w.mapAddressBook.count(a));
        CHECK_EQ(w.mapAddressBook[a].name, std::string("alice"));
        CHECK_EQ(w.mapAddressBook[a].purpose, std::string("receive"));
        std::string v;
        CHECK(w.GetDestData(a, "rr0", &v) && v == "request-0");
        CHECK(!w.GetDestData(a, "used", &v));
        CHECK(!w.mapAddressBook.count(b));
        CHECK(!w.GetDestData(b, "rr1", &v));
    }
    std::string cmd = std::string("rm -rf '") + tmpl + "'";
    CHECK(std::system(cmd.c_str()) == 0);
}

namespace {
// A Berkeley DB 4.x btree file as the reference's wallet.dat has it (a master database listing
// the sub-database "main", whose tree is an internal page over leaf pages, big items in overflow
// chains), written from the page layout of db_page.h. No libdb exists here to write a real one,
// so this pins the reader against that layout only.
struct BdbWriter {
    explicit BdbWriter(size_t pagesize) : P(pagesize) {}
    size_t P;
    std::vector<std::string> pages;
    static void put16(std::string& pg, size_t off, uint32_t v) {
        pg[off] = (char)(v & 0xff);
        pg[off + 1] = (char)((v >> 8) & 0xff);
    }
    static void put32(std::string& pg, size_t off, uint32_t v) {
        for (int i = 0; i < 4; i++) pg[off + i] = (char)((v >> (8 * i)) & 0xff);
    }
    uint32_t NewPage(uint8_t type) {
        pages.emplace_back(P, '\0');
        const uint32_t pg = (uint32_t)pages.size() - 1;
        put32(pages[pg], 8, pg);
        pages[pg][25] = (char)type;
        return pg;
    }
    void Meta(uint32_t pg, uint32_t root, bool subdbs) {
        std::string& m = pages[pg];
        put32(m, 12, 0x053162);
        put32(m, 16, 9); // btree version
        put32(m, 20, (uint32_t)P);
        m[25] = 9;
        put32(m, 48, subdbs ? 0x20 : 0);
        put32(m, 88, root);
    }
    // item bytes: inline B_KEYDATA, or a B_OVERFLOW reference to a new overflow chain
    std::string Item(const std::string& v) {
        if (3 + v.size() <= P / 4) {
            std::string it(3, '\0');
            put16(it, 0, (uint32_t)v.size());
            it[2] = 1;
            return it + v;
        }
        uint32_t first = 0, prev = 0;
        for (size_t off = 0; off < v.size(); off += P - 26) {
            const uint32_t pg = NewPage(7);
            const size_t len = std::min(P - 26, v.size() - off);
            put16(pages[pg], 22, (uint32_t)len);
            pages[pg].replace(26, len, v.substr(off, len));
            if (off == 0) first = pg;
            else put32(pages[prev], 16, pg);
            prev = pg;
        }
        std::string it(12, '\0');
        it[2] = 3;
        put32(it, 4, first);
        put32(it, 8, (uint32_t)v.size());
        return it;
    }
    // leaf pages of (key, value) pairs; returns their page numbers
    std::vector<uint32_t> Leaves(const std::vector<std::pair<std::string, std::string>>& recs) {
        std::vector<uint32_t> leaves;
        uint32_t pg = 0;
        size_t n = 0, top = P;
        for (const auto& kv : recs) {
            const std::string a = Item(kv.first), b = Item(kv.second);
            if (!leaves.size() || 26 + 2 * (n + 2) + (a.size() + b.size()) > top) {
                pg = NewPage(5);
                leaves.push_back(pg);
                n = 0;
                top = P;
            }
            for (const std::string* it : {&a, &b}) {
                top -= it->size();
                pages[pg].replace(top, it->size(), *it);
                put16(pages[pg], 26 + 2 * n, (uint32_t)top);
                put16(pages[pg], 20, (uint32_t)++n);
            }
        }
        return leaves;
    }
    uint32_t Internal(const std::vector<uint32_t>& children) {
        const uint32_t pg = NewPage(3);
        size_t top = P;
        for (size_t i = 0; i < children.size(); i++) {
            std::string it(12, '\0');
            it[2] = 1;
            put32(it, 4, children[i]);
            top -= it.size();
            pages[pg].replace(top, it.size(), it);
            put16(pages[pg], 26 + 2 * i, (uint32_t)top);
        }
        put16(pages[pg], 20, (uint32_t)children.size());
        pages[pg][24] = 2; // level
        return pg;
    }
    std::string File(const std::vector<std::pair<std::string, std::string>>& recs) {
        NewPage(9); // 0: master meta
        const uint32_t mleaf = NewPage(5), smeta = NewPage(9);
        const std::vector<uint32_t> leaves = Leaves(recs);
        const uint32_t root = Internal(leaves);
        Meta(smeta, root, false);
        // master leaf: "main" -> the sub-database's meta page
        std::string pg4(4, '\0');
        put32(pg4, 0, smeta);
        const std::string a = Item("main"), b = Item(pg4);
        pages[mleaf].replace(P - a.size(), a.size(), a);
        pages[mleaf].replace(P - a.size() - b.size(), b.size(), b);
        put16(pages[mleaf], 26, (uint32_t)(P - a.size()));
        put16(pages[mleaf], 28, (uint32_t)(P - a.size() - b.size()));
        put16(pages[mleaf], 20, 2);
        Meta(0, mleaf, true);
        put32(pages[0], 32, (uint32_t)pages.size() - 1); // last_pgno
        std::string f;
        for (const auto& p : pages) f += p;
        return f;
    }
};

std::string HexOf(const std::string& s) {
    static const char* d = "0123456789abcdef";
    std::string o;
    for (unsigned char c : s) {
        o += d[c >> 4];
        o += d[c & 15];
    }
    return o;
}
} // namespace

// A wallet's records written as a reference wallet.dat (BDB btree file, and db_dump text) are
// imported by the loader's conversion and load back with the same keys, names and data.
TEST_CASE(walletdb_tests, bdb_wallet_import) {
    char tmpl[] = "/tmp/bcp_bdbimport_XXXXXX";
    REQUIRE(mkdtemp(tmpl) != nullptr);
    const std::string dir = tmpl;
    std::set<CKeyID> keys;
    CKey k;
    k.MakeNewKey(true);
    const CTxDestination a = k.GetPubKey().GetID();
    const std::string big(6000, 'z'); // an overflow item in a 4 KiB page file
    {
        CWallet w("src", dir + "/src", false);
        std::string err;
        bool first = false;
        REQUIRE(w.Load(err, first));
        REQUIRE(w.SetHDMasterKey(w.GenerateNewHDMasterKey()));
        REQUIRE(w.TopUpKeyPool(30));
        CHECK(w.SetAddressBook(a, "alice", "receive"));
        CHECK(w.AddDestData(a, "rr0", big));
        keys = w.GetKeys();
        w.Flush();
    }
    REQUIRE(keys.size() >= 30);
    std::vector<std::pair<std::string, std::string>> recs;
    {
        KVStore db(dir + "/src", false, false);
        KVIterator it(&db);
        for (it.SeekToFirst(); it.Valid(); it.Next()) {
            std::string v;
            it.RawValue(v);
            recs.emplace_back(it.RawKey(), v);
        }
    }
    REQUIRE(recs.size() > 60);
    // unencrypted keys as the reference writes them: the DER SEC1 ECPrivateKey (version 1, the
    // secret, tagged curve parameters, the public key) plus a trailing 32-byte hash
    size_t nKeyRecs = 0;
    for (auto& kv : recs) {
        SpanReader kr((const unsigned char*)kv.first.data(), kv.first.size(), SER_DISK, PROTOCOL_VERSION);
        std::string type;
        kr >> type;
        if (type != "key") continue;
        CPubKey pub;
        kr >> pub;
        SpanReader vr((const unsigned char*)kv.second.data(), kv.second.size(), SER_DISK, PROTOCOL_VERSION);
        std::vector<unsigned char> secret;
        vr >> secret;
        REQUIRE(secret.size() == 32);
        std::vector<unsigned char> inner = {0x02, 0x01, 0x01, 0x04, 0x20};
        inner.insert(inner.end(), secret.begin(), secret.end());
        const std::vector<unsigned char> params = {0xa0, 0x03, 0x06, 0x01, 0x00};
        inner.insert(inner.end(), params.begin(), params.end());
        inner.push_back(0xa1);
        inner.push_back((unsigned char)(pub.size() + 3));
        inner.push_back(0x03);
        inner.push_back((unsigned char)(pub.size() + 1));
        inner.push_back(0x00);
        inner.insert(inner.end(), pub.begin(), pub.end());
        std::vector<unsigned char> der = {0x30, 0x81, (unsigned char)inner.size()};
        der.insert(der.end(), inner.begin(), inner.end());
        std::vector<unsigned char> v;
        VectorWriter w(v, SER_DISK, PROTOCOL_VERSION);
        w << der << uint256();
        kv.second.assign(v.begin(), v.end());
        nKeyRecs++;
    }
    REQUIRE(nKeyRecs >= 30);
    // the btree file
    {
        std::ofstream f(dir + "/wallet.dat", std::ios::binary);
        const std::string bytes = BdbWriter(4096).File(recs);
        f.write(bytes.data(), bytes.size());
    }
    BdbRecords got;
    std::string err;
    REQUIRE(ReadBdbBtree(dir + "/wallet.dat", got, err));
    CHECK(got == recs);
    CHECK_EQ(BdbFileKind(dir + "/wallet.dat"), std::string("btree"));
    size_t n = 0;
    REQUIRE(ImportBdbWalletFile(dir + "/wallet.dat", n, err));
    CHECK_EQ(n, recs.size());
    CHECK(BdbFileKind(dir + "/wallet.dat").empty()); // now this wallet's store
    {
        CWallet w("wallet.dat", dir + "/wallet.dat", false);
        bool first = true;
        REQUIRE(w.Load(err, first));
        CHECK(!first);
        CHECK(w.GetKeys() == keys);
        CHECK(w.IsHDEnabled());
        CHECK_EQ(w.mapAddressBook[a].name, std::string("alice"));
        std::string v;
        CHECK(w.GetDestData(a, "rr0", &v) && v == big);
    }
    // the db_dump text of the same records
    {
        std::ofstream f(dir + "/dump.dat");
        f << "VERSION=3\nformat=bytevalue\ndatabase=main\ntype=btree\ndb_pagesize=4096\nHEADER=END\n";
        for (const auto& kv : recs) f << " " << HexOf(kv.first) << "\n " << HexOf(kv.second) << "\n";
        f << "DATA=END\n";
    }
    CHECK_EQ(BdbFileKind(dir + "/dump.dat"), std::string("dump"));
    REQUIRE(ImportBdbWalletFile(dir + "/dump.dat", n, err));
    CHECK_EQ(n, recs.size());
    {
        CWallet w("dump.dat", dir + "/dump.dat", false);
        bool first = true;
        REQUIRE(w.Load(err, first));
        CHECK(w.GetKeys() == keys);
    }
    // damaged files fail cleanly
    {
        std::string bytes = BdbWriter(4096).File(recs);
        std::ofstream(dir + "/trunc.dat", std::ios::binary).write(bytes.data(), 4096 * 3);
        CHECK(!ReadBdbBtree(dir + "/trunc.dat", got, err));
        for (size_t i = 4096; i < bytes.size(); i += 97) bytes[i] = (char)(bytes[i] ^ 0x5a); // scribble on every page
        std::ofstream(dir + "/bad.dat", std::ios::binary).write(bytes.data(), bytes.size());
        got.clear();
        ReadBdbBtree(dir + "/bad.dat", got, err); // any verdict, but bounded and no crash
        std::istringstream dump("VERSION=3\nHEADER=END\n 00\nDATA=END\n");
        CHECK(!ReadBdbDump(dump, got, err)); // a key without a value
    }
    std::string cmd = "rm -rf '" + dir + "'";
    CHECK(std::system(cmd.c_str()) == 0);
}

} // namespace bcp
