// Python bindings: script parsing, interpreter, signature hashing, standard templates
// and signing. The DoTest harness mirrors reference src/test/script_tests.cpp:119-200
// (crediting + spending transaction around the tested scripts).
#include "python/bind.h"
#include "script/interpreter.h"
#include "script/sign.h"
#include "script/standard.h"
#include "consensus/tx_verify.h"

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
}

} // namespace py
} // namespace bcp
