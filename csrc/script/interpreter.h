// Script interpreter: flags, errors, FORKID signature digest, signature checkers.
// Behaviour parity with reference src/script/interpreter.{h,cpp}:
//   flag bits                      interpreter.h:32-120 (incl. SCRIPT_ALLOW_NON_FORKID)
//   CheckSignatureEncoding         interpreter.cpp:222-256 (ILLEGAL/MUST_USE_FORKID)
//   EvalScript                     interpreter.cpp:299-1320 (disabled opcodes :344-353)
//   SignatureHash (FORKID/BIP143)  interpreter.cpp:1354-1404, legacy :1406-1428
//   VerifyScript                   interpreter.cpp:1550-1629
//   script_error names             src/script/script_error.cpp / test/script_tests.cpp:54-92
//
// Batch-verification design (MI355X): a DeferringSignatureChecker can record ECDSA
// checks instead of executing them. This is sound exactly when NULLFAIL is active
// and the signature is non-empty: a failing CHECKSIG then fails the whole script,
// so "assume true now, verify later in a GPU batch, AND the results" yields the same
// accept/reject decision. CHECKMULTISIG, where a failed (signature, key) pair is legal, is
// deferred speculatively under the same NULLFAIL condition: every pair the greedy match could
// try goes into the batch, and the match itself is replayed over the batch results
// (DeferredMultisig / EvalDeferredMultisig). Non-NULLFAIL contexts are evaluated eagerly.
#pragma once
#include "kernels/gpu_api.h"
#include "primitives/transaction.h"
#include "script/script.h"

#include <cstring>
#include <string>
#include <vector>

namespace bcp {

enum {
    SIGHASH_ALL = 1,
    SIGHASH_NONE = 2,
    SIGHASH_SINGLE = 3,
    SIGHASH_FORKID = 0x40,
    SIGHASH_ANYONECANPAY = 0x80,
};

enum : uint32_t {
    SCRIPT_VERIFY_NONE = 0,
    SCRIPT_VERIFY_P2SH = (1U << 0),
    SCRIPT_VERIFY_STRICTENC = (1U << 1),
    SCRIPT_VERIFY_DERSIG = (1U << 2),
    SCRIPT_VERIFY_LOW_S = (1U << 3),
    SCRIPT_VERIFY_NULLDUMMY = (1U << 4),
    SCRIPT_VERIFY_SIGPUSHONLY = (1U << 5),
    SCRIPT_VERIFY_MINIMALDATA = (1U << 6),
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS = (1U << 7),
    SCRIPT_VERIFY_CLEANSTACK = (1U << 8),
    SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY = (1U << 9),
    SCRIPT_VERIFY_CHECKSEQUENCEVERIFY = (1U << 10),
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM = (1U << 12),
    SCRIPT_VERIFY_MINIMALIF = (1U << 13),
    SCRIPT_VERIFY_NULLFAIL = (1U << 14),
    SCRIPT_VERIFY_COMPRESSED_PUBKEYTYPE = (1U << 15),
    SCRIPT_ENABLE_SIGHASH_FORKID = (1U << 16),
    SCRIPT_ALLOW_NON_FORKID = (1U << 17),
};

// Policy flag sets (reference src/script/standard.h:43, src/policy/policy.h:60-75).
static const uint32_t MANDATORY_SCRIPT_VERIFY_FLAGS = SCRIPT_VERIFY_P2SH | SCRIPT_VERIFY_STRICTENC |
                                                      SCRIPT_ENABLE_SIGHASH_FORKID | SCRIPT_VERIFY_LOW_S |
                                                      SCRIPT_VERIFY_NULLFAIL;
static const uint32_t STANDARD_SCRIPT_VERIFY_FLAGS =
    MANDATORY_SCRIPT_VERIFY_FLAGS | SCRIPT_VERIFY_DERSIG | SCRIPT_VERIFY_MINIMALDATA | SCRIPT_VERIFY_NULLDUMMY |
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS | SCRIPT_VERIFY_CLEANSTACK | SCRIPT_VERIFY_NULLFAIL |
    SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY | SCRIPT_VERIFY_CHECKSEQUENCEVERIFY | SCRIPT_VERIFY_LOW_S |
    SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM;
static const uint32_t STANDARD_NOT_MANDATORY_VERIFY_FLAGS = STANDARD_SCRIPT_VERIFY_FLAGS & ~MANDATORY_SCRIPT_VERIFY_FLAGS;

enum ScriptError {
    SCRIPT_ERR_OK = 0,
    SCRIPT_ERR_UNKNOWN_ERROR,
    SCRIPT_ERR_EVAL_FALSE,
    SCRIPT_ERR_OP_RETURN,
    SCRIPT_ERR_SCRIPT_SIZE,
    SCRIPT_ERR_PUSH_SIZE,
    SCRIPT_ERR_OP_COUNT,
    SCRIPT_ERR_STACK_SIZE,
    SCRIPT_ERR_SIG_COUNT,
    SCRIPT_ERR_PUBKEY_COUNT,
    SCRIPT_ERR_VERIFY,
    SCRIPT_ERR_EQUALVERIFY,
    SCRIPT_ERR_CHECKMULTISIGVERIFY,
    SCRIPT_ERR_CHECKSIGVERIFY,
    SCRIPT_ERR_NUMEQUALVERIFY,
    SCRIPT_ERR_BAD_OPCODE,
    SCRIPT_ERR_DISABLED_OPCODE,
    SCRIPT_ERR_INVALID_STACK_OPERATION,
    SCRIPT_ERR_INVALID_ALTSTACK_OPERATION,
    SCRIPT_ERR_UNBALANCED_CONDITIONAL,
    SCRIPT_ERR_NEGATIVE_LOCKTIME,
    SCRIPT_ERR_UNSATISFIED_LOCKTIME,
    SCRIPT_ERR_SIG_HASHTYPE,
    SCRIPT_ERR_SIG_DER,
    SCRIPT_ERR_MINIMALDATA,
    SCRIPT_ERR_SIG_PUSHONLY,
    SCRIPT_ERR_SIG_HIGH_S,
    SCRIPT_ERR_SIG_NULLDUMMY,
    SCRIPT_ERR_PUBKEYTYPE,
    SCRIPT_ERR_CLEANSTACK,
    SCRIPT_ERR_MINIMALIF,
    SCRIPT_ERR_SIG_NULLFAIL,
    SCRIPT_ERR_DISCOURAGE_UPGRADABLE_NOPS,
    SCRIPT_ERR_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM,
    SCRIPT_ERR_NONCOMPRESSED_PUBKEY,
    SCRIPT_ERR_ILLEGAL_FORKID,
    SCRIPT_ERR_MUST_USE_FORKID,
    SCRIPT_ERR_ERROR_COUNT
};

const char* ScriptErrorString(ScriptError err);   // human-readable (RPC reject reasons)
const char* ScriptErrorName(ScriptError err);     // short test-vector name ("EVAL_FALSE", ...)
bool ParseScriptErrorName(const std::string& name, ScriptError& out);
uint32_t ParseScriptFlags(const std::string& commaList); // "P2SH,STRICTENC"; throws on unknown
std::string FormatScriptFlags(uint32_t flags);

bool CastToBool(const std::vector<unsigned char>& vch);
bool CheckSignatureEncoding(const std::vector<unsigned char>& vchSig, uint32_t flags, ScriptError* serror);
bool IsValidSignatureEncoding(const std::vector<unsigned char>& sig); // strict DER (BIP66)

uint256 SignatureHash(const CScript& scriptCode, const CTransaction& txTo, unsigned int nIn, uint32_t nHashType,
                      Amount amount, const PrecomputedTransactionData* cache = nullptr,
                      uint32_t flags = SCRIPT_ENABLE_SIGHASH_FORKID);

class BaseSignatureChecker {
public:
    virtual ~BaseSignatureChecker() {}
    // `deferrable` is true when a false result is guaranteed to fail the script
    // (NULLFAIL + non-empty signature, CHECKSIG/CHECKSIGVERIFY): a batching checker
    // may record the check and return true.
    virtual bool CheckSig(const std::vector<unsigned char>& sig, const std::vector<unsigned char>& pubkey,
                          const CScript& scriptCode, uint32_t flags, bool deferrable = false) const {
        return false;
    }
    // CHECKMULTISIG under NULLFAIL with only non-empty, well-encoded signatures (a failed match
    // then fails the script): a batching checker may record the match for later and return
    // true. keyOk bit j: key j passes the key-encoding rules (a visited bad key fails the script).
    virtual bool DeferMultisig(const std::vector<const std::vector<unsigned char>*>& sigs,
                               const std::vector<const std::vector<unsigned char>*>& keys, uint32_t keyOk,
                               const CScript& scriptCode, uint32_t flags) const {
        return false;
    }
    virtual bool CheckLockTime(const CScriptNum& nLockTime) const { return false; }
    virtual bool CheckSequence(const CScriptNum& nSequence) const { return false; }
};

class TransactionSignatureChecker : public BaseSignatureChecker {
public:
    TransactionSignatureChecker(const CTransaction* txTo, unsigned int nIn, Amount amount,
                                const PrecomputedTransactionData* txdata = nullptr)
        : txTo(txTo), nIn(nIn), amount(amount), txdata(txdata) {}
    bool CheckSig(const std::vector<unsigned char>& sig, const std::vector<unsigned char>& pubkey,
                  const CScript& scriptCode, uint32_t flags, bool deferrable = false) const override;
    bool CheckLockTime(const CScriptNum& nLockTime) const override;
    bool CheckSequence(const CScriptNum& nSequence) const override;

protected:
    // Digest for a signature with its hashtype byte (memoised); false if the signature is empty.
    bool SigDigest(const std::vector<unsigned char>& sigIn, const CScript& scriptCode, uint32_t flags,
                   uint256& sighash) const;
    // Computes the digest and splits off the hashtype; false if the signature is empty.
    bool PrepareSig(const std::vector<unsigned char>& sigIn, const CScript& scriptCode, uint32_t flags,
                    std::vector<unsigned char>& sigOut, uint256& sighash) const;
    virtual bool VerifySignature(const std::vector<unsigned char>& sig, const std::vector<unsigned char>& pubkey,
                                 const uint256& sighash) const;
    const CTransaction* txTo;
    unsigned int nIn;
    Amount amount;
    const PrecomputedTransactionData* txdata;

private:
    // Last digest computed by this checker: a script that checks signatures repeatedly under the
    // same script code and hash type (e.g. a P2SH redeem script of many CHECKSIGVERIFYs) hashes
    // the transaction once instead of once per check.
    mutable CScript memoCode;
    mutable uint32_t memoHashType = 0, memoFlags = 0;
    mutable bool memoValid = false;
    mutable uint256 memoSighash;
};

// Fixed-capacity byte string stored inline: a block's deferred checks (up to ~200k) are created
// on the script workers and freed together after the batch, without two heap blocks each.
template <size_t CAP> struct InlineBytes {
    static constexpr size_t capacity = CAP;
    uint8_t len = 0;
    unsigned char buf[CAP];
    const unsigned char* data() const { return buf; }
    size_t size() const { return len; }
    const unsigned char* begin() const { return buf; }
    const unsigned char* end() const { return buf + len; }
    unsigned char operator[](size_t i) const { return buf[i]; }
    bool assign(const unsigned char* p, size_t n) {
        if (n > CAP) return false;
        memcpy(buf, p, n);
        len = (uint8_t)n;
        return true;
    }
    bool assign(const std::vector<unsigned char>& v) { return assign(v.data(), v.size()); }
};

// One ECDSA verification recorded for later batch execution (GPU).
struct DeferredSigCheck {
    InlineBytes<65> pubkey; // serialized (33/65 bytes)
    InlineBytes<72> sig;    // DER (strict DER is at most 72 bytes), hashtype stripped
    uint256 sighash; // the signature hash (computed by the script worker that deferred the check)
};

// A deferred CHECKMULTISIG: the m x (n - m + 1) pairs its greedy match can reach are consecutive
// checks of the batch starting at `first`, row-major by signature (signature i with keys
// i .. i + n - m). Their individual results are speculative: only the replayed match counts.
struct DeferredMultisig {
    uint32_t first = 0; // index of the first pair check (rebased when job sinks are concatenated)
    uint8_t m = 0, n = 0;
    uint32_t keyOk = 0; // bit j: key j passes the key-encoding rules
    uint32_t Pairs() const { return (uint32_t)m * (uint32_t)(n - m + 1); }
};
// Replays the reference's greedy CHECKMULTISIG loop (interpreter.cpp:1054) over the pair results.
bool EvalDeferredMultisig(const DeferredMultisig& g, const uint8_t* pairResults);

class DeferringSignatureChecker : public TransactionSignatureChecker {
public:
    DeferringSignatureChecker(const CTransaction* txTo, unsigned int nIn, Amount amount,
                              const PrecomputedTransactionData* txdata, std::vector<DeferredSigCheck>* sink,
                              std::vector<DeferredMultisig>* groups = nullptr)
        : TransactionSignatureChecker(txTo, nIn, amount, txdata), sink(sink), groups(groups) {}
    bool CheckSig(const std::vector<unsigned char>& sig, const std::vector<unsigned char>& pubkey,
                  const CScript& scriptCode, uint32_t flags, bool deferrable = false) const override;
    bool DeferMultisig(const std::vector<const std::vector<unsigned char>*>& sigs,
                       const std::vector<const std::vector<unsigned char>*>& keys, uint32_t keyOk,
                       const CScript& scriptCode, uint32_t flags) const override;
private:
    std::vector<DeferredSigCheck>* sink;
    std::vector<DeferredMultisig>* groups; // CHECKMULTISIG deferral (null: multisig runs eagerly)
};

class MutableTransactionSignatureChecker : public TransactionSignatureChecker {
public:
    MutableTransactionSignatureChecker(const CMutableTransaction* txTo, unsigned int nIn, Amount amount)
        : TransactionSignatureChecker(&tx, nIn, amount), tx(*txTo) {}

private:
    const CTransaction tx;
};

bool EvalScript(std::vector<std::vector<unsigned char>>& stack, const CScript& script, uint32_t flags,
                const BaseSignatureChecker& checker, ScriptError* error = nullptr);
bool VerifyScript(const CScript& scriptSig, const CScript& scriptPubKey, uint32_t flags,
                  const BaseSignatureChecker& checker, ScriptError* serror = nullptr);

} // namespace bcp
