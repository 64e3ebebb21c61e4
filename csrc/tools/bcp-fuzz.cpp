// bcp-fuzz: deserialization fuzz harness (reference src/test/test_bitcoin_fuzzy.cpp:29-47 and
// doc/fuzzing.md). Reads one input from stdin (or the files named on the command line, one
// input each): the first 4 bytes (little endian) pick a target, the rest is the payload. Every
// target parses untrusted bytes the way the node does and exercises what the node then does
// with the object (hashing, round-trip re-serialization, validity checks); malformed input
// must end in a caught deserialization error, never a crash, hang or assertion. Works as an
// AFL/libFuzzer-style stdin harness and is driven by tests/test_fuzz.py.
//
//   bcp-fuzz [-target=<name>] [file...]   (-target=<name> skips the 4-byte selector)
//   bcp-fuzz -list
#include "consensus/chain.h"
#include "consensus/merkle.h"
#include "consensus/params.h"
#include "consensus/pow.h"
#include "consensus/equihash.h"
#include "consensus/merkleblock.h"
#include "consensus/tx_verify.h"
#include "crypto/hashes.h"
#include "consensus/validation_state.h"
#include "net/addrman.h"
#include "net/blockencodings.h"
#include "net/netaddress.h"
#include "net/protocol.h"
#include "node/coins.h"
#include "primitives/block.h"
#include "primitives/transaction.h"
#include "script/interpreter.h"
#include "script/standard.h"
#include "util/util.h"

#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <functional>
#include <iostream>
#include <iterator>
#include <map>
#include <string>
#include <vector>

using namespace bcp;

namespace {

typedef std::vector<unsigned char> Bytes;

// Round trip: whatever parsed must re-serialize to a prefix of the input it came from.
template <typename T> void RoundTrip(const T& obj, const Bytes& in, size_t consumed, int version) {
    Bytes out;
    VectorWriter w(out, SER_NETWORK, version);
    w << obj;
    if (out.size() != consumed || memcmp(out.data(), in.data(), consumed) != 0) {
        // non-canonical encodings (e.g. oversized CompactSize) may legitimately differ; the
        // re-serialized form must at least parse back to itself
        T again;
        SpanReader r(out.data(), out.size(), SER_NETWORK, version);
        r >> again;
        Bytes out2;
        VectorWriter w2(out2, SER_NETWORK, version);
        w2 << again;
        if (out2 != out) {
            fprintf(stderr, "round trip mismatch\n");
            abort();
        }
    }
}

template <typename T> bool Parse(const Bytes& in, T& obj, int version = PROTOCOL_VERSION, int type = SER_NETWORK,
                                 size_t* consumed = nullptr) {
    try {
        SpanReader r(in.data(), in.size(), type, version);
        r >> obj;
        if (consumed) *consumed = in.size() - r.size();
        return true;
    } catch (const std::ios_base::failure&) {
        return false;
    }
}

const CChainParams& Main() {
    static bool init = false;
    if (!init) {
        SelectParams("main");
        init = true;
    }
    return Params();
}

std::map<std::string, std::function<void(const Bytes&)>>& Targets() {
    static std::map<std::string, std::function<void(const Bytes&)>> t;
    return t;
}
struct Reg {
    Reg(const char* name, std::function<void(const Bytes&)> f) { Targets()[name] = f; }
};

void BlockTarget(const Bytes& in, int version) {
    CBlock block;
    size_t used = 0;
    if (!Parse(in, block, version, SER_NETWORK, &used)) return;
    (void)block.GetHash(Main().GetConsensus());
    // the context-free checks CheckBlock applies to every received block
    CValidationState state;
    bool mutated = false;
    (void)BlockMerkleRoot(block, &mutated);
    (void)GetSerializeSize(block, version);
    if (!block.vtx.empty()) {
        (void)CheckCoinbase(*block.vtx[0], state, false);
        for (size_t i = 1; i < block.vtx.size(); ++i) (void)CheckRegularTransaction(*block.vtx[i], state, false);
    }
    RoundTrip(block, in, used, version);
}

Reg r_block("block", [](const Bytes& in) { BlockTarget(in, PROTOCOL_VERSION); });
Reg r_block_legacy("block_legacy", [](const Bytes& in) { BlockTarget(in, PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY); });

Reg r_header("block_header", [](const Bytes& in) {
    CBlockHeader h;
    size_t used = 0;
    if (!Parse(in, h, PROTOCOL_VERSION, SER_NETWORK, &used)) return;
    (void)h.GetHash(Main().GetConsensus());
    // the Equihash check runs on attacker-controlled solutions in every headers message
    (void)CheckEquihashSolution(&h, Main());
    RoundTrip(h, in, used, PROTOCOL_VERSION);
});

Reg r_tx("transaction", [](const Bytes& in) {
    CMutableTransaction mtx;
    size_t used = 0;
    if (!Parse(in, mtx, PROTOCOL_VERSION, SER_NETWORK, &used)) return;
    const CTransaction tx(mtx);
    (void)tx.GetHash();
    CValidationState state;
    (void)CheckRegularTransaction(tx, state);
    (void)CheckCoinbase(tx, state);
    for (const CTxOut& out : tx.vout) {
        txnouttype type;
        std::vector<std::vector<unsigned char>> sol;
        (void)Solver(out.scriptPubKey, type, sol);
    }
    RoundTrip(mtx, in, used, PROTOCOL_VERSION);
});

Reg r_locator("block_locator", [](const Bytes& in) {
    CBlockLocator l;
    (void)Parse(in, l);
});

Reg r_disk_index("disk_block_index", [](const Bytes& in) {
    CDiskBlockIndex d;
    if (!Parse(in, d, CLIENT_VERSION, SER_DISK)) return;
    (void)d.GetBlockHash();
});

Reg r_coin("coin", [](const Bytes& in) {
    Coin c;
    (void)Parse(in, c, CLIENT_VERSION, SER_DISK);
});
Reg r_txundo("tx_undo", [](const Bytes& in) {
    CTxUndo u;
    (void)Parse(in, u, CLIENT_VERSION, SER_DISK);
});
Reg r_blockundo("block_undo", [](const Bytes& in) {
    CBlockUndo u;
    (void)Parse(in, u, CLIENT_VERSION, SER_DISK);
});

Reg r_address("address", [](const Bytes& in) {
    CAddress a;
    if (!Parse(in, a)) return;
    (void)a.IsRoutable();
    (void)a.GetGroup();
    (void)a.ToStringIPPort();
});
Reg r_inv("inv", [](const Bytes& in) {
    CInv i;
    if (Parse(in, i)) (void)i.ToString();
});
Reg r_msg_header("message_header", [](const Bytes& in) {
    CMessageHeader h;
    if (Parse(in, h)) (void)h.IsValid(Main().NetMagic());
});

Reg r_bloom("bloom_filter", [](const Bytes& in) {
    CBloomFilter f;
    if (!Parse(in, f)) return;
    if (!f.IsWithinSizeConstraints()) return;
    f.UpdateEmptyFull();
    (void)f.contains(uint256());
    (void)f.contains(Bytes{1, 2, 3});
});
Reg r_pmt("partial_merkle_tree", [](const Bytes& in) {
    CPartialMerkleTree t;
    if (!Parse(in, t)) return;
    std::vector<uint256> matches;
    std::vector<unsigned> idx;
    (void)t.ExtractMatches(matches, idx);
});
Reg r_merkleblock("merkle_block", [](const Bytes& in) {
    CMerkleBlock mb;
    if (!Parse(in, mb)) return;
    std::vector<uint256> matches;
    std::vector<unsigned> idx;
    (void)mb.txn.ExtractMatches(matches, idx);
});

Reg r_cmpct("cmpct_block", [](const Bytes& in) {
    CBlockHeaderAndShortTxIDs c;
    if (!Parse(in, c)) return;
    (void)c.BlockTxCount();
});
Reg r_getblocktxn("block_transactions_request", [](const Bytes& in) {
    BlockTransactionsRequest r;
    (void)Parse(in, r);
});
Reg r_blocktxn("block_transactions", [](const Bytes& in) {
    BlockTransactions b;
    (void)Parse(in, b);
});

Reg r_addrman("addrman", [](const Bytes& in) {
    // peers.dat framing: magic || payload || SHA256d checksum, parsed from a temp file
    Bytes file(Main().NetMagic(), Main().NetMagic() + 4);
    file.insert(file.end(), in.begin(), in.end());
    const uint256 sum = Hash256(file.data(), file.size());
    file.insert(file.end(), sum.begin(), sum.end());
    char path[] = "/tmp/bcp-fuzz-addrmanXXXXXX";
    const int fd = mkstemp(path);
    if (fd < 0) return;
    if (write(fd, file.data(), file.size()) != (ssize_t)file.size()) {
        close(fd);
        unlink(path);
        return;
    }
    close(fd);
    CAddrMan am;
    (void)am.Read(path, Main().NetMagic());
    (void)am.size();
    unlink(path);
});

Reg r_script("script_eval", [](const Bytes& in) {
    // first 4 bytes: verify flags; rest: a script run with a checker that rejects signatures
    if (in.size() < 4) return;
    uint32_t flags;
    memcpy(&flags, in.data(), 4);
    const CScript script(in.begin() + 4, in.end());
    std::vector<std::vector<unsigned char>> stack;
    BaseSignatureChecker checker;
    ScriptError err;
    (void)EvalScript(stack, script, flags, checker, &err);
    (void)script.IsPushOnly();
    (void)script.IsPayToScriptHash();
});

Reg r_equihash("equihash_solution", [](const Bytes& in) {
    // header-free Equihash check on (48,5) and (200,9): raw input = solution bytes
    for (auto nk : {std::make_pair(48u, 5u), std::make_pair(200u, 9u)}) {
        const EquihashParams p(nk.first, nk.second);
        CBlake2b st = EhInitialiseState(p);
        st.Write(in.data(), std::min<size_t>(in.size(), 140));
        std::string why;
        (void)EhIsValidSolution(p, st, in, &why);
    }
});

} // namespace

int main(int argc, char* argv[]) {
    std::string forced;
    std::vector<std::string> files;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "-list") {
            for (const auto& t : Targets()) printf("%s\n", t.first.c_str());
            return 0;
        }
        if (a.rfind("-target=", 0) == 0) forced = a.substr(8);
        else files.push_back(a);
    }
    if (!forced.empty() && !Targets().count(forced)) {
        fprintf(stderr, "unknown target %s\n", forced.c_str());
        return 2;
    }
    std::vector<std::string> names;
    for (const auto& t : Targets()) names.push_back(t.first);
    auto run = [&](const Bytes& buf) {
        if (!forced.empty()) {
            Targets()[forced](buf);
            return;
        }
        if (buf.size() < 4) return;
        uint32_t sel;
        memcpy(&sel, buf.data(), 4);
        const Bytes payload(buf.begin() + 4, buf.end());
        Targets()[names[sel % names.size()]](payload);
    };
    if (files.empty()) {
        const Bytes buf((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
        run(buf);
    } else {
        for (const std::string& f : files) {
            FILE* fp = fopen(f.c_str(), "rb");
            if (!fp) continue;
            Bytes buf;
            unsigned char tmp[65536];
            size_t n;
            while ((n = fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.insert(buf.end(), tmp, tmp + n);
            fclose(fp);
            run(buf);
        }
    }
    return 0;
}
