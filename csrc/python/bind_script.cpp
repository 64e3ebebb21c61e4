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
#include "script/sighash_recipe.h"
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

    // FORKID signature-hash recipes (K7): items = [(script_code, tx, n_in, hash_type, amount)].
    // Returns [(digest, recipe_used)]: the device (use_gpu) or CPU evaluation of each recipe;
    // checks the recipe cannot express (legacy, SIGHASH_SINGLE with a matching output) carry the
    // CPU SignatureHash as a PRECOMPUTED job.
    m.def(
        "sighash_recipes",
        [](const std::vector<std::tuple<pyb::bytes, pyb::bytes, unsigned, uint32_t, int64_t>>& items, bool use_gpu,
           uint32_t flags, int device) {
            const size_t n = items.size();
            std::vector<gpu::SighashTx> txs(n);
            std::vector<gpu::SighashJob> jobs(n);
            std::vector<unsigned char> code, pre(n * 32, 0);
            std::vector<bool> used(n);
            for (size_t i = 0; i < n; i++) {
                const CScript sc = to_script(std::get<0>(items[i]));
                const CTransaction tx = tx_from_bytes(std::get<1>(items[i]));
                const unsigned nIn = std::get<2>(items[i]);
                const uint32_t ht = std::get<3>(items[i]);
                const Amount amount = std::get<4>(items[i]);
                if (nIn >= tx.vin.size()) throw std::invalid_argument("n_in out of range");
                const PrecomputedTransactionData txdata(tx);
                FillSighashTx(tx, txdata, txs[i]);
                used[i] = FillSighashJob(tx, nIn, ht, amount, flags, (uint32_t)i, (uint32_t)code.size(),
                                         (uint32_t)sc.size(), jobs[i]);
                if (used[i]) {
                    code.insert(code.end(), sc.begin(), sc.end());
                } else {
                    memset(&jobs[i], 0, sizeof(jobs[i]));
                    jobs[i].flags = gpu::SIGHASH_JOB_PRECOMPUTED;
                    const uint256 h = SignatureHash(sc, tx, nIn, ht, amount, &txdata, flags);
                    memcpy(&pre[32 * i], h.begin(), 32);
                }
            }
            std::vector<unsigned char> out(n * 32);
            if (use_gpu) {
                pyb::gil_scoped_release rel;
                out = gpu::SighashBatch(txs, jobs, code, pre, device);
            } else {
                for (size_t i = 0; i < n; i++) {
                    const uint256 h = used[i] ? SighashFromRecipe(txs[i], jobs[i], code.data()) : uint256();
                    memcpy(&out[32 * i], used[i] ? h.begin() : &pre[32 * i], 32);
                }
            }
            pyb::list l;
            for (size_t i = 0; i < n; i++) l.append(pyb::make_tuple(to_bytes(&out[32 * i], 32), (bool)used[i]));
            return l;
        },
        pyb::arg("items"), pyb::arg("use_gpu") = false, pyb::arg("flags") = (uint32_t)SCRIPT_ENABLE_SIGHASH_FORKID,
        pyb::arg("device") = -1);

    // Block-validation signature checks through the node's deferral path with device sighash
    // recipes (DeferringSignatureChecker::SetRecipes): items = [(pubkey, sig_with_hashtype,
    // script_code, tx, n_in, amount)]. The GPU path is the fused digest -> verify lane batch
    // (GpuVerifyDeferred); the CPU path evaluates each recipe (DeferredDigest) and verifies.
    // Returns (results, digests, recipe flags); a check the checker refused to defer is (False,
    // b"", False).
    m.def(
        "verify_sig_recipes",
        [](const std::vector<std::tuple<pyb::bytes, pyb::bytes, pyb::bytes, pyb::bytes, unsigned, int64_t>>& items,
           bool use_gpu, bool recipes, uint32_t flags) {
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
                checker.SetRecipes(recipes);
                const size_t before = sink.size();
                checker.CheckSig(to_vec(std::get<1>(items[i])), to_vec(std::get<0>(items[i])),
                                 to_script(std::get<2>(items[i])), flags, true);
                if (sink.size() > before) slot[i] = (int)before;
            }
            std::vector<const DeferredSigCheck*> ptrs;
            for (const auto& c : sink) ptrs.push_back(&c);
            std::vector<uint8_t> res(sink.size());
            std::vector<uint256> dg(sink.size());
            {
                pyb::gil_scoped_release rel;
                if (use_gpu && !sink.empty()) {
                    res = GpuVerifyDeferred(ptrs, nullptr, &dg);
                } else {
                    for (size_t j = 0; j < sink.size(); j++) {
                        const DeferredSigCheck& c = sink[j];
                        dg[j] = DeferredDigest(c);
                        res[j] = secp::VerifySignature(c.pubkey.data(), c.pubkey.size(), c.sig.data(), c.sig.size(),
                                                       dg[j].begin());
                    }
                }
            }
            pyb::list r, d, f;
            for (size_t i = 0; i < n; i++) {
                if (slot[i] < 0) {
                    r.append(false);
                    d.append(pyb::bytes(""));
                    f.append(false);
                    continue;
                }
                r.append((bool)res[slot[i]]);
                d.append(to_bytes(dg[slot[i]].begin(), 32));
                f.append(sink[slot[i]].recipe);
            }
            return pyb::make_tuple(r, d, f);
        },
        pyb::arg("items"), pyb::arg("use_gpu") = false, pyb::arg("recipes") = true,
        pyb::arg("flags") = (uint32_t)(SCRIPT_ENABLE_SIGHASH_FORKID | SCRIPT_VERIFY_STRICTENC));
}

} // namespace py
} // namespace bcp
