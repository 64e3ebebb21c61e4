// Python bindings: consensus data model (chain params, headers/blocks/txs, merkle,
// difficulty), secp256k1/keys and address encodings. Used by the unit tests and
// by the Python tooling; the node itself runs entirely in C++.
#include "consensus/chain.h"
#include "crypto/common.h"
#include "consensus/merkle.h"
#include "consensus/params.h"
#include "consensus/pow.h"
#include "keys/key.h"
#include "primitives/block.h"
#include "primitives/transaction.h"
#include "python/bind.h"
#include "secp256k1/secp256k1.h"

#include <deque>
#include <memory>

namespace bcp {
namespace py {

static uint256 u256_from_bytes(const pyb::bytes& b) {
    std::vector<unsigned char> v = to_vec(b);
    if (v.size() != 32) throw std::invalid_argument("expected 32 bytes");
    uint256 r;
    memcpy(r.begin(), v.data(), 32);
    return r;
}
static pyb::bytes u256_bytes(const uint256& u) { return to_bytes(u.begin(), 32); }

// A growable chain of CBlockIndex entries for difficulty tests: blocks are appended
// with a time delta and nBits; chain work accumulates as in the reference test
// helper (src/test/pow_tests.cpp:100-112).
class ChainSim {
public:
    explicit ChainSim(const std::string& chain) : params(&Params(chain)) {}
    void add(int64_t time_or_delta, uint32_t bits, bool absolute) {
        blocks.emplace_back();
        CBlockIndex& b = blocks.back();
        hashes.emplace_back();
        hashes.back().SetNull();
        WriteLE32(hashes.back().begin(), (uint32_t)blocks.size());
        b.phashBlock = &hashes.back();
        if (blocks.size() == 1) {
            b.pprev = nullptr;
            b.nHeight = start_height;
            b.nTime = (uint32_t)time_or_delta;
            b.nBits = bits;
            b.nChainWork = GetBlockProof(b);
        } else {
            CBlockIndex* prev = &blocks[blocks.size() - 2];
            b.pprev = prev;
            b.nHeight = prev->nHeight + 1;
            b.nTime = absolute ? (uint32_t)time_or_delta : (uint32_t)((int64_t)prev->nTime + time_or_delta);
            b.nBits = bits;
            b.nChainWork = prev->nChainWork + GetBlockProof(b);
        }
        if (start_height == 0) b.BuildSkip(); // partial chains: ancestors below start do not exist
    }
    uint32_t next_work(int64_t header_time) const {
        CBlockHeader h;
        h.nTime = (uint32_t)header_time;
        return GetNextWorkRequired(tip(), &h, params->GetConsensus());
    }
    uint32_t cashplus_next_work(int64_t header_time) const {
        CBlockHeader h;
        h.nTime = (uint32_t)header_time;
        return GetNextCashPlusWorkRequired(tip(), &h, params->GetConsensus());
    }
    const CBlockIndex* tip() const { return blocks.empty() ? nullptr : &blocks.back(); }
    int height() const { return blocks.empty() ? -1 : blocks.back().nHeight; }
    int64_t median_time_past() const { return tip() ? tip()->GetMedianTimePast() : 0; }
    std::string chain_work_hex() const { return tip() ? tip()->nChainWork.GetHex() : std::string(); }
    int start_height = 0;

private:
    const CChainParams* params;
    std::deque<CBlockIndex> blocks; // deque: stable addresses for pprev
    std::deque<uint256> hashes;
};

static pyb::dict header_to_dict(const CBlockHeader& h) {
    pyb::dict d;
    d["version"] = h.nVersion;
    d["prev"] = h.hashPrevBlock.GetHex();
    d["merkle_root"] = h.hashMerkleRoot.GetHex();
    d["height"] = h.nHeight;
    d["time"] = h.nTime;
    d["bits"] = h.nBits;
    d["nonce"] = h.nNonce.GetHex();
    d["solution"] = to_bytes(h.nSolution);
    return d;
}

void bind_consensus(pyb::module_& m) {
    // ---------------------------------------------------------------- chain params
    m.def("chain_params", [](const std::string& chain) {
        const CChainParams& p = Params(chain);
        const Consensus::Params& c = p.GetConsensus();
        pyb::dict d;
        d["network"] = p.NetworkIDString();
        d["genesis_hash"] = c.hashGenesisBlock.GetHex();
        d["genesis_merkle_root"] = p.GenesisBlock().hashMerkleRoot.GetHex();
        d["net_magic"] = to_bytes(p.NetMagic(), 4);
        d["disk_magic"] = to_bytes(p.DiskMagic(), 4);
        d["port"] = p.GetDefaultPort();
        d["rpc_port"] = p.GetRPCPort();
        d["equihash_n"] = p.EquihashN();
        d["equihash_k"] = p.EquihashK();
        d["bcp_height"] = c.BCPHeight;
        d["bcp_premine_window"] = c.BCPPremineWindow;
        d["pow_limit"] = c.powLimit.GetHex();
        d["pow_limit_legacy"] = c.powLimitLegacy.GetHex();
        d["pow_limit_start"] = c.powLimitStart.GetHex();
        d["pow_averaging_window"] = c.nPowAveragingWindow;
        d["pow_target_spacing"] = c.nPowTargetSpacing;
        d["no_retargeting"] = c.fPowNoRetargeting;
        d["allow_min_difficulty"] = c.fPowAllowMinDifficultyBlocks;
        d["cashaddr_prefix"] = p.CashAddrPrefix();
        d["pubkey_prefix"] = to_bytes(p.Base58Prefix(CChainParams::PUBKEY_ADDRESS));
        d["script_prefix"] = to_bytes(p.Base58Prefix(CChainParams::SCRIPT_ADDRESS));
        d["secret_prefix"] = to_bytes(p.Base58Prefix(CChainParams::SECRET_KEY));
        d["halving_interval"] = c.nSubsidyHalvingInterval;
        d["anti_replay_sunset"] = c.antiReplayOpReturnSunsetHeight;
        d["anti_replay_commitment"] = to_bytes(c.antiReplayOpReturnCommitment);
        pyb::dict cps;
        for (const auto& kv : p.Checkpoints().mapCheckpoints) cps[pyb::int_(kv.first)] = kv.second.GetHex();
        d["checkpoints"] = cps;
        return d;
    });
    m.def("genesis_block", [](const std::string& chain) {
        return to_bytes(SerializeToBytes(Params(chain).GenesisBlock(), SER_NETWORK,
                                         PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY));
    });
    m.def("block_subsidy", [](int height, const std::string& chain) {
        return GetBlockSubsidy(height, Params(chain).GetConsensus());
    });
    m.def("select_params", [](const std::string& chain) { SelectParams(chain); });

    // ---------------------------------------------------------------- headers / blocks / txs
    m.def(
        "header_decode",
        [](const pyb::bytes& b, bool legacy) {
            std::vector<unsigned char> v = to_vec(b);
            SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0));
            CBlockHeader h;
            r >> h;
            return header_to_dict(h);
        },
        pyb::arg("data"), pyb::arg("legacy") = false);
    m.def(
        "header_hash",
        [](const pyb::bytes& b, bool legacy, const std::string& chain) {
            std::vector<unsigned char> v = to_vec(b);
            SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0));
            CBlockHeader h;
            r >> h;
            return h.GetHash(Params(chain).GetConsensus()).GetHex();
        },
        pyb::arg("data"), pyb::arg("legacy") = false, pyb::arg("chain") = "main");
    m.def(
        "block_decode",
        [](const pyb::bytes& b, bool legacy, const std::string& chain) {
            std::vector<unsigned char> v = to_vec(b);
            SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0));
            CBlock blk;
            r >> blk;
            pyb::dict d = header_to_dict(blk);
            d["hash"] = blk.GetHash(Params(chain).GetConsensus()).GetHex();
            pyb::list txids;
            for (const auto& tx : blk.vtx) txids.append(tx->GetHash().GetHex());
            d["txids"] = txids;
            bool mutated = false;
            d["computed_merkle_root"] = BlockMerkleRoot(blk, &mutated).GetHex();
            d["mutated"] = mutated;
            d["reserialized"] = to_bytes(SerializeToBytes(
                blk, SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0)));
            return d;
        },
        pyb::arg("data"), pyb::arg("legacy") = false, pyb::arg("chain") = "main");
    m.def("equihash_input", [](const pyb::bytes& b) {
        std::vector<unsigned char> v = to_vec(b);
        SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
        CBlockHeader h;
        r >> h;
        return to_bytes(h.EquihashInput());
    });
    m.def("check_equihash_header", [](const pyb::bytes& b, const std::string& chain) {
        std::vector<unsigned char> v = to_vec(b);
        SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
        CBlockHeader h;
        r >> h;
        return CheckEquihashSolution(&h, Params(chain));
    });
    // Batched header check (CheckEquihashSolutions): GPU for >= 4 headers, CPU fallback on device errors.
    m.def(
        "check_equihash_headers",
        [](const std::vector<pyb::bytes>& hs, const std::string& chain, bool allow_gpu) {
            std::vector<CBlockHeader> headers(hs.size());
            for (size_t i = 0; i < hs.size(); ++i) {
                std::vector<unsigned char> v = to_vec(hs[i]);
                SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
                r >> headers[i];
            }
            std::vector<const CBlockHeader*> ptrs;
            for (auto& h : headers) ptrs.push_back(&h);
            pyb::gil_scoped_release nogil;
            return CheckEquihashSolutions(ptrs, Params(chain), allow_gpu);
        },
        pyb::arg("headers"), pyb::arg("chain") = "regtest", pyb::arg("allow_gpu") = true);
    m.def("tx_decode", [](const pyb::bytes& b) {
        std::vector<unsigned char> v = to_vec(b);
        SpanReader r(v.data(), v.size(), SER_NETWORK, PROTOCOL_VERSION);
        CMutableTransaction mtx;
        r >> mtx;
        CTransaction tx(mtx);
        pyb::dict d;
        d["txid"] = tx.GetHash().GetHex();
        d["version"] = tx.nVersion;
        d["locktime"] = tx.nLockTime;
        pyb::list vin, vout;
        for (const auto& in : tx.vin) {
            pyb::dict i;
            i["prev_txid"] = in.prevout.hash.GetHex();
            i["prev_n"] = in.prevout.n;
            i["script_sig"] = to_bytes(std::vector<unsigned char>(in.scriptSig.begin(), in.scriptSig.end()));
            i["sequence"] = in.nSequence;
            vin.append(i);
        }
        for (const auto& out : tx.vout) {
            pyb::dict o;
            o["value"] = out.nValue;
            o["script_pubkey"] = to_bytes(std::vector<unsigned char>(out.scriptPubKey.begin(), out.scriptPubKey.end()));
            vout.append(o);
        }
        d["vin"] = vin;
        d["vout"] = vout;
        d["is_coinbase"] = tx.IsCoinBase();
        d["reserialized"] = to_bytes(SerializeToBytes(tx));
        return d;
    });

    // ---------------------------------------------------------------- merkle
    m.def("merkle_root", [](const std::vector<pyb::bytes>& leaves) {
        std::vector<uint256> v;
        for (const auto& l : leaves) v.push_back(u256_from_bytes(l));
        bool mutated = false;
        uint256 r = ComputeMerkleRoot(v, &mutated);
        return pyb::make_tuple(u256_bytes(r), mutated);
    });
    m.def("merkle_branch", [](const std::vector<pyb::bytes>& leaves, uint32_t pos) {
        std::vector<uint256> v;
        for (const auto& l : leaves) v.push_back(u256_from_bytes(l));
        std::vector<pyb::bytes> out;
        for (const auto& h : ComputeMerkleBranch(v, pos)) out.push_back(u256_bytes(h));
        return out;
    });
    m.def("merkle_root_from_branch", [](const pyb::bytes& leaf, const std::vector<pyb::bytes>& branch, uint32_t idx) {
        std::vector<uint256> v;
        for (const auto& l : branch) v.push_back(u256_from_bytes(l));
        return u256_bytes(ComputeMerkleRootFromBranch(u256_from_bytes(leaf), v, idx));
    });
    m.def("set_gpu_merkle_threshold", &SetGpuMerkleThreshold);

    // ---------------------------------------------------------------- difficulty
    pyb::class_<ChainSim>(m, "ChainSim")
        .def(pyb::init<const std::string&>())
        .def_readwrite("start_height", &ChainSim::start_height)
        .def("add", &ChainSim::add, pyb::arg("time"), pyb::arg("bits"), pyb::arg("absolute") = false)
        .def("next_work", &ChainSim::next_work, pyb::arg("header_time") = 0)
        .def("cashplus_next_work", &ChainSim::cashplus_next_work, pyb::arg("header_time") = 0)
        .def_property_readonly("height", &ChainSim::height)
        .def_property_readonly("median_time_past", &ChainSim::median_time_past)
        .def_property_readonly("chain_work", &ChainSim::chain_work_hex);
    m.def("calculate_next_work", [](int height, uint32_t time, uint32_t bits, int64_t first_time, const std::string& chain) {
        CBlockIndex idx;
        idx.nHeight = height;
        idx.nTime = time;
        idx.nBits = bits;
        return CalculateNextWorkRequired(&idx, first_time, Params(chain).GetConsensus());
    });
    m.def("check_proof_of_work", [](const std::string& hash_hex, uint32_t bits, bool postfork, const std::string& chain) {
        return CheckProofOfWork(uint256S(hash_hex), bits, postfork, Params(chain).GetConsensus());
    });
    m.def("block_proof_hex", [](uint32_t bits) {
        CBlockIndex idx;
        idx.nBits = bits;
        return GetBlockProof(idx).GetHex();
    });

    // ---------------------------------------------------------------- secp256k1 / keys
    m.def("ec_seckey_verify", [](const pyb::bytes& k) {
        auto v = to_vec(k);
        return v.size() == 32 && secp::seckey_verify(v.data());
    });
    m.def(
        "ec_pubkey_create",
        [](const pyb::bytes& k, bool compressed) {
            auto v = to_vec(k);
            CKey key;
            key.Set(v.begin(), v.end(), compressed);
            if (!key.IsValid()) throw std::invalid_argument("invalid secret key");
            return to_bytes(key.GetPubKey().Raw());
        },
        pyb::arg("seckey"), pyb::arg("compressed") = true);
    m.def(
        "ec_sign",
        [](const pyb::bytes& k, const pyb::bytes& msg, uint32_t test_case) {
            auto v = to_vec(k);
            CKey key;
            key.Set(v.begin(), v.end(), true);
            if (!key.IsValid()) throw std::invalid_argument("invalid secret key");
            std::vector<unsigned char> sig;
            key.Sign(u256_from_bytes(msg), sig, test_case);
            return to_bytes(sig);
        },
        pyb::arg("seckey"), pyb::arg("msg32"), pyb::arg("test_case") = 0);
    m.def(
        "ec_sign_compact",
        [](const pyb::bytes& k, const pyb::bytes& msg, bool compressed) {
            auto v = to_vec(k);
            CKey key;
            key.Set(v.begin(), v.end(), compressed);
            if (!key.IsValid()) throw std::invalid_argument("invalid secret key");
            std::vector<unsigned char> sig;
            key.SignCompact(u256_from_bytes(msg), sig);
            return to_bytes(sig);
        },
        pyb::arg("seckey"), pyb::arg("msg32"), pyb::arg("compressed") = true);
    m.def("ec_recover_compact", [](const pyb::bytes& msg, const pyb::bytes& sig) -> pyb::object {
        CPubKey pk;
        if (!pk.RecoverCompact(u256_from_bytes(msg), to_vec(sig))) return pyb::none();
        return to_bytes(pk.Raw());
    });
    m.def("ec_verify", [](const pyb::bytes& pub, const pyb::bytes& sig, const pyb::bytes& msg) {
        auto p = to_vec(pub), s = to_vec(sig);
        uint256 h = u256_from_bytes(msg);
        return secp::VerifySignature(p.data(), p.size(), s.data(), s.size(), h.begin());
    });
    m.def("ec_check_low_s", [](const pyb::bytes& sig) { return CPubKey::CheckLowS(to_vec(sig)); });
    m.def("ec_pubkey_valid", [](const pyb::bytes& pub) { return CPubKey(to_vec(pub)).IsFullyValid(); });
    m.def("ec_pubkey_decompress", [](const pyb::bytes& pub) -> pyb::object {
        CPubKey pk(to_vec(pub));
        if (!pk.Decompress()) return pyb::none();
        return to_bytes(pk.Raw());
    });
    m.def("ec_rfc6979_nonce", [](const pyb::bytes& msg, const pyb::bytes& key, pyb::object extra, unsigned counter) {
        auto mm = to_vec(msg), kk = to_vec(key);
        std::vector<unsigned char> ee;
        if (!extra.is_none()) ee = to_vec(extra.cast<pyb::bytes>());
        unsigned char out[32];
        secp::rfc6979_nonce(out, mm.data(), kk.data(), ee.empty() ? nullptr : ee.data(), counter);
        return to_bytes(out, 32);
    });
    m.def("ec_seckey_tweak_add", [](const pyb::bytes& k, const pyb::bytes& t) -> pyb::object {
        auto kk = to_vec(k), tt = to_vec(t);
        if (!secp::seckey_tweak_add(kk.data(), tt.data())) return pyb::none();
        return to_bytes(kk);
    });

    // ---------------------------------------------------------------- encodings
    m.def("base58_encode", [](const pyb::bytes& b) { return EncodeBase58(to_vec(b)); });
    m.def("base58_decode", [](const std::string& s) -> pyb::object {
        std::vector<unsigned char> v;
        if (!DecodeBase58(s, v)) return pyb::none();
        return to_bytes(v);
    });
    m.def("base58check_encode", [](const pyb::bytes& b) { return EncodeBase58Check(to_vec(b)); });
    m.def("base58check_decode", [](const std::string& s) -> pyb::object {
        std::vector<unsigned char> v;
        if (!DecodeBase58Check(s, v)) return pyb::none();
        return to_bytes(v);
    });
    m.def("cashaddr_encode", [](const std::string& prefix, const std::vector<uint8_t>& values) {
        return cashaddr::Encode(prefix, values);
    });
    m.def("cashaddr_decode", [](const std::string& s, const std::string& default_prefix) {
        auto r = cashaddr::Decode(s, default_prefix);
        return pyb::make_tuple(r.first, r.second);
    });
    m.def(
        "encode_destination",
        [](const std::string& kind, const pyb::bytes& h, const std::string& chain, pyb::object cash) {
            auto v = to_vec(h);
            if (v.size() != 20) throw std::invalid_argument("hash must be 20 bytes");
            uint160 u;
            memcpy(u.begin(), v.data(), 20);
            CTxDestination d = kind == "script" ? CTxDestination(CScriptID(u)) : CTxDestination(CKeyID(u));
            const CChainParams& p = Params(chain);
            if (cash.is_none()) return EncodeDestination(d, p);
            return cash.cast<bool>() ? EncodeCashAddr(d, p) : EncodeLegacyAddr(d, p);
        },
        pyb::arg("kind"), pyb::arg("hash160"), pyb::arg("chain") = "main", pyb::arg("cashaddr") = pyb::none());
    m.def(
        "decode_destination",
        [](const std::string& s, const std::string& chain) -> pyb::object {
            CTxDestination d = DecodeDestination(s, Params(chain));
            if (!d.IsValid()) return pyb::none();
            return pyb::make_tuple(d.type == DestType::KEYID ? "pubkey" : "script", to_bytes(d.hash.begin(), 20));
        },
        pyb::arg("addr"), pyb::arg("chain") = "main");
    m.def("set_use_cashaddr", &SetUseCashAddr);
    m.def(
        "encode_secret",
        [](const pyb::bytes& k, bool compressed, const std::string& chain) {
            auto v = to_vec(k);
            CKey key;
            key.Set(v.begin(), v.end(), compressed);
            if (!key.IsValid()) throw std::invalid_argument("invalid secret key");
            return EncodeSecret(key, Params(chain));
        },
        pyb::arg("seckey"), pyb::arg("compressed") = true, pyb::arg("chain") = "main");
    m.def(
        "decode_secret",
        [](const std::string& s, const std::string& chain) -> pyb::object {
            CKey key = DecodeSecret(s, Params(chain));
            if (!key.IsValid()) return pyb::none();
            return pyb::make_tuple(to_bytes(key.GetPrivKeyBytes()), key.IsCompressed());
        },
        pyb::arg("wif"), pyb::arg("chain") = "main");
    m.def(
        "bip32_master",
        [](const pyb::bytes& seed, const std::string& chain) {
            auto s = to_vec(seed);
            CExtKey k;
            k.SetMaster(s.data(), (unsigned)s.size());
            return pyb::make_tuple(EncodeExtKey(k, Params(chain)), EncodeExtPubKey(k.Neuter(), Params(chain)));
        },
        pyb::arg("seed"), pyb::arg("chain") = "main");
    m.def(
        "bip32_derive",
        [](const std::string& xprv, uint32_t child, const std::string& chain) {
            CExtKey k = DecodeExtKey(xprv, Params(chain));
            if (!k.key.IsValid()) throw std::invalid_argument("bad xprv");
            CExtKey out;
            if (!k.Derive(out, child)) throw std::runtime_error("derivation failed");
            return pyb::make_tuple(EncodeExtKey(out, Params(chain)), EncodeExtPubKey(out.Neuter(), Params(chain)));
        },
        pyb::arg("xprv"), pyb::arg("child"), pyb::arg("chain") = "main");
    m.def(
        "bip32_derive_pub",
        [](const std::string& xpub, uint32_t child, const std::string& chain) {
            CExtPubKey k = DecodeExtPubKey(xpub, Params(chain));
            if (!k.pubkey.IsValid()) throw std::invalid_argument("bad xpub");
            CExtPubKey out;
            if (!k.Derive(out, child)) throw std::runtime_error("derivation failed");
            return EncodeExtPubKey(out, Params(chain));
        },
        pyb::arg("xpub"), pyb::arg("child"), pyb::arg("chain") = "main");
    m.def("message_hash", [](const std::string& msg) { return u256_bytes(MessageHash(msg)); });
}

} // namespace py
} // namespace bcp
