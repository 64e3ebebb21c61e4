// Python bindings: script parsing, interpreter, signature hashing, standard templates
// and signing. The DoTest harness mirrors reference src/test/script_tests.cpp:119-200
// (crediting + spending transaction around the tested scripts).
#include "python/bind.h"
#include "script/interpreter.h"
#include "script/sign.h"
#include "script/standard.h"
#include "consensus/tx_verify.h"
#include "kernels/gpu_api.h"
#include "node/sigverify.h"
#include "secp256k1/secp256k1.h"

#include <cstring>
#include <memory>

namespace bcp {
namespace py {

static CScript to_script(const pyb::bytes& b) {
    auto v = to_vec(b);
    return CScript(v.begin(), v.end());
}
static pyb::bytes script_bytes(const CScript& s) { return to_bytes(std::vector<unsigned char>(s.begin(), s.end())); }

static CTransaction tx_from_bytes(const pyb::bytes& b) {
    auto v = to_vec(b);
    SpanReader r(v.data(), v.size());
    CMutableTransaction m;
    r >> m;
    return CTransaction(m);
}

void bind_script(pyb::module_& m) {
    m.def("parse_script", [](const std::string& s) { return script_bytes(ParseScript(s)); });
    m.def(
        "script_to_asm",
        [](const pyb::bytes& b, bool sighash_decode) { return ScriptToAsmStr(to_script(b), sighash_decode); },
        pyb::arg("script"), pyb::arg("sighash_decode") = false);
    m.def("parse_script_flags", &ParseScriptFlags);
    m.def("format_script_flags", &FormatScriptFlags);
    m.def("script_error_name", [](int e) { return std::string(ScriptErrorName((ScriptError)e)); });
    m.attr("STANDARD_SCRIPT_VERIFY_FLAGS") = STANDARD_SCRIPT_VERIFY_FLAGS;
    m.attr("MANDATORY_SCRIPT_VERIFY_FLAGS") = MANDATORY_SCRIPT_VERIFY_FLAGS;

    // (ok, error_name) for the script_tests.json harness.
    m.def("script_test", [](const pyb::bytes& sig, const pyb::bytes& spk, uint32_t flags, int64_t amount) {
        const CScript scriptSig = to_script(sig), scriptPubKey = to_script(spk);
        if (flags & SCRIPT_VERIFY_CLEANSTACK) flags |= SCRIPT_VERIFY_P2SH;
        CMutableTransaction credit;
        credit.nVersion = 1;
        credit.nLockTime = 0;
        credit.vin.resize(1);
        credit.vout.resize(1);
        credit.vin[0].prevout.SetNull();
        credit.vin[0].scriptSig = CScript() << CScriptNum(0) << CScriptNum(0);
        credit.vin[0].nSequence = CTxIn::SEQUENCE_FINAL;
        credit.vout[0].scriptPubKey = scriptPubKey;
        credit.vout[0].nValue = amount;
        CMutableTransaction spend;
        spend.nVersion = 1;
        spend.nLockTime = 0;
        spend.vin.resize(1);
        spend.vout.resize(1);
        spend.vin[0].prevout.hash = credit.GetId();
        spend.vin[0].prevout.n = 0;
        spend.vin[0].scriptSig = scriptSig;
        spend.vin[0].nSequence = CTxIn::SEQUENCE_FINAL;
        spend.vout[0].scriptPubKey = CScript();
        spend.vout[0].nValue = amount;
        ScriptError err;
        MutableTransactionSignatureChecker checker(&spend, 0, amount);
        const bool ok = VerifyScript(scriptSig, scriptPubKey, flags, checker, &err);
        return pyb::make_tuple(ok, std::string(ScriptErrorName(err)));
    });
    m.def(
        "verify_tx_input",
        [](const pyb::bytes& txb, unsigned nIn, const pyb::bytes& spk, int64_t amount, uint32_t flags) {
            CTransaction tx = tx_from_bytes(txb);
            if (nIn >= tx.vin.size()) throw std::out_of_range("input index");
            PrecomputedTransactionData txdata(tx);
            TransactionSignatureChecker checker(&tx, nIn, amount, &txdata);
            ScriptError err;
            const bool ok = VerifyScript(tx.vin[nIn].scriptSig, to_script(spk), flags, checker, &err);
            return pyb::make_tuple(ok, std::string(ScriptErrorName(err)));
        },
        pyb::arg("tx"), pyb::arg("n_in"), pyb::arg("script_pubkey"), pyb::arg("amount") = 0,
        pyb::arg("flags") = STANDARD_SCRIPT_VERIFY_FLAGS);
    m.def(
        "signature_hash",
        [](const pyb::bytes& code, const pyb::bytes& txb, unsigned nIn, uint32_t ht, int64_t amount, uint32_t flags) {
            CTransaction tx = tx_from_bytes(txb);
            uint256 h = SignatureHash(to_script(code), tx, nIn, ht, amount, nullptr, flags);
            return to_bytes(h.begin(), 32);
        },
        pyb::arg("script_code"), pyb::arg("tx"), pyb::arg("n_in"), pyb::arg("hash_type"), pyb::arg("amount") = 0,
        pyb::arg("flags") = (uint32_t)SCRIPT_ENABLE_SIGHASH_FORKID);
    m.def("check_transaction", [](const pyb::bytes& txb) {
        CTransaction tx = tx_from_bytes(txb);
        CValidationState st;
        const bool ok = tx.IsCoinBase() ? CheckCoinbase(tx, st) : CheckRegularTransaction(tx, st);
        return pyb::make_tuple(ok, st.GetRejectReason());
    });
    m.def("solver", [](const pyb::bytes& spk) {
        txnouttype t;
        std::vector<std::vector<unsigned char>> sol;
        Solver(to_script(spk), t, sol);
        std::vector<pyb::bytes> out;
        for (auto& s : sol) out.push_back(to_bytes(s));
        return pyb::make_tuple(std::string(GetTxnOutputType(t)), out);
    });
    m.def("script_for_destination", [](const std::string& kind, const pyb::bytes& h) {
        auto v = to_vec(h);
        if (v.size() != 20) throw std::invalid_argument("hash160 expected");
        uint160 u(v);
        return script_bytes(GetScriptForDestination(kind == "script" ? CTxDestination(CScriptID(u))
                                                                      : CTxDestination(CKeyID(u))));
    });
    m.def("script_for_multisig", [](int n, const std::vector<pyb::bytes>& keys) {
        std::vector<CPubKey> pks;
        for (auto& k : keys) pks.emplace_back(to_vec(k));
        return script_bytes(GetScriptForMultisig(n, pks));
    });
    // Sign input nIn of tx spending `spk` with the given secret keys (and redeem scripts).
    m.def(
        "sign_tx_input",
        [](const pyb::bytes& txb, unsigned nIn, const pyb::bytes& spk, int64_t amount,
           const std::vector<std::pair<pyb::bytes, bool>>& keys, const std::vector<pyb::bytes>& redeem, uint32_t ht) {
            auto v = to_vec(txb);
            SpanReader r(v.data(), v.size());
            CMutableTransaction mtx;
            r >> mtx;
            CBasicKeyStore ks;
            for (auto& k : keys) {
                auto kb = to_vec(k.first);
                CKey key;
                key.Set(kb.begin(), kb.end(), k.second);
                if (!key.IsValid()) throw std::invalid_argument("invalid key");
                ks.AddKey(key);
            }
            for (auto& rs : redeem) ks.AddCScript(to_script(rs));
            const bool ok = SignSignature(ks, to_script(spk), mtx, nIn, amount, ht);
            return pyb::make_tuple(ok, to_bytes(SerializeToBytes(mtx)));
        },
        pyb::arg("tx"), pyb::arg("n_in"), pyb::arg("script_pubkey"), pyb::arg("amount"), pyb::arg("keys"),
        pyb::arg("redeem_scripts") = std::vector<pyb::bytes>(), pyb::arg("hash_type") = SIGHASH_ALL | SIGHASH_FORKID);

    // Block-validation signature checks through the node's deferral path: items = [(pubkey,
    // sig_with_hashtype, script_code, tx, n_in, amount)]. Each check's digest is computed by the
    // deferring checker (as a script worker does); the GPU path is the verify lane batch
    // (GpuVerifyDeferred), the CPU path verifies each check. Returns (results, digests); a check
    // the checker refused to defer is (False, b"").
    m.def(
        "verify_sig_deferred",
        [](const std::vector<std::tuple<pyb::bytes, pyb::bytes, pyb::bytes, pyb::bytes, unsigned, int64_t>>& items,
           bool use_gpu, uint32_t flags) {
            const size_t n = items.size();
            std::vector<std::unique_ptr<CTransaction>> txs;
            std::vector<std::unique_ptr<PrecomputedTransactionData>> txdatas;
            std::vector<DeferredSigCheck> sink;
            std::vector<int> slot(n, -1);
            for (size_t i = 0; i < n; i++) {
                txs.emplace_back(new CTransaction(tx_from_bytes(std::get<3>(items[i]))));
                txdatas.emplace_back(new PrecomputedTransactionData(*txs.back()));
                const unsigned nIn = std::get<4>(items[i]);
                if (nIn >= txs.back()->vin.size()) throw std::invalid_argument("n_in out of range");
                DeferringSignatureChecker checker(txs.back().get(), nIn, std::get<5>(items[i]), txdatas.back().get(),
                                                  &sink);
                const size_t before = sink.size();
                checker.CheckSig(to_vec(std::get<1>(items[i])), to_vec(std::get<0>(items[i])),
                                 to_script(std::get<2>(items[i])), flags, true);
                if (sink.size() > before) slot[i] = (int)before;
            }
            std::vector<const DeferredSigCheck*> ptrs;
            for (const auto& c : sink) ptrs.push_back(&c);
            std::vector<uint8_t> res(sink.size());
            {
                pyb::gil_scoped_release rel;
                if (use_gpu && !sink.empty()) {
                    res = GpuVerifyDeferred(ptrs);
                } else {
                    for (size_t j = 0; j < sink.size(); j++) {
                        const DeferredSigCheck& c = sink[j];
                        res[j] = secp::VerifySignature(c.pubkey.data(), c.pubkey.size(), c.sig.data(), c.sig.size(),
                                                       c.sighash.begin());
                    }
                }
            }
            pyb::list r, d;
            for (size_t i = 0; i < n; i++) {
                if (slot[i] < 0) {
                    r.append(false);
                    d.append(pyb::bytes(""));
                    continue;
                }
                r.append((bool)res[slot[i]]);
                d.append(to_bytes(sink[slot[i]].sighash.begin(), 32));
            }
            return pyb::make_tuple(r, d);
        },
        pyb::arg("items"), pyb::arg("use_gpu") = false,
        pyb::arg("flags") = (uint32_t)(SCRIPT_ENABLE_SIGHASH_FORKID | SCRIPT_VERIFY_STRICTENC));
}

} // namespace py
} // namespace bcp
