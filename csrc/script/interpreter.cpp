// Script interpreter. See interpreter.h for the parity map.
#include "script/interpreter.h"
#include "crypto/hashes.h"
#include "keys/key.h"
#include "secp256k1/secp256k1.h"

#include <algorithm>
#include <cstring>
#include <map>

namespace bcp {

typedef std::vector<unsigned char> valtype;

// ------------------------------------------------------------------ error names
namespace {
struct ErrInfo {
    ScriptError e;
    const char* name;
    const char* text;
};
const ErrInfo kErrors[] = {
    {SCRIPT_ERR_OK, "OK", "No error"},
    {SCRIPT_ERR_UNKNOWN_ERROR, "UNKNOWN_ERROR", "unknown error"},
    {SCRIPT_ERR_EVAL_FALSE, "EVAL_FALSE", "Script evaluated without error but finished with a false/empty top stack element"},
    {SCRIPT_ERR_OP_RETURN, "OP_RETURN", "OP_RETURN was encountered"},
    {SCRIPT_ERR_SCRIPT_SIZE, "SCRIPT_SIZE", "Script is too big"},
    {SCRIPT_ERR_PUSH_SIZE, "PUSH_SIZE", "Push value size limit exceeded"},
    {SCRIPT_ERR_OP_COUNT, "OP_COUNT", "Operation limit exceeded"},
    {SCRIPT_ERR_STACK_SIZE, "STACK_SIZE", "Stack size limit exceeded"},
    {SCRIPT_ERR_SIG_COUNT, "SIG_COUNT", "Signature count negative or greater than pubkey count"},
    {SCRIPT_ERR_PUBKEY_COUNT, "PUBKEY_COUNT", "Pubkey count negative or limit exceeded"},
    {SCRIPT_ERR_VERIFY, "VERIFY", "Script failed an OP_VERIFY operation"},
    {SCRIPT_ERR_EQUALVERIFY, "EQUALVERIFY", "Script failed an OP_EQUALVERIFY operation"},
    {SCRIPT_ERR_CHECKMULTISIGVERIFY, "CHECKMULTISIGVERIFY", "Script failed an OP_CHECKMULTISIGVERIFY operation"},
    {SCRIPT_ERR_CHECKSIGVERIFY, "CHECKSIGVERIFY", "Script failed an OP_CHECKSIGVERIFY operation"},
    {SCRIPT_ERR_NUMEQUALVERIFY, "NUMEQUALVERIFY", "Script failed an OP_NUMEQUALVERIFY operation"},
    {SCRIPT_ERR_BAD_OPCODE, "BAD_OPCODE", "Opcode missing or not understood"},
    {SCRIPT_ERR_DISABLED_OPCODE, "DISABLED_OPCODE", "Attempted to use a disabled opcode"},
    {SCRIPT_ERR_INVALID_STACK_OPERATION, "INVALID_STACK_OPERATION", "Operation not valid with the current stack size"},
    {SCRIPT_ERR_INVALID_ALTSTACK_OPERATION, "INVALID_ALTSTACK_OPERATION", "Operation not valid with the current altstack size"},
    {SCRIPT_ERR_UNBALANCED_CONDITIONAL, "UNBALANCED_CONDITIONAL", "Invalid OP_IF construction"},
    {SCRIPT_ERR_NEGATIVE_LOCKTIME, "NEGATIVE_LOCKTIME", "Negative locktime"},
    {SCRIPT_ERR_UNSATISFIED_LOCKTIME, "UNSATISFIED_LOCKTIME", "Locktime requirement not satisfied"},
    {SCRIPT_ERR_SIG_HASHTYPE, "SIG_HASHTYPE", "Signature hash type missing or not understood"},
    {SCRIPT_ERR_SIG_DER, "SIG_DER", "Non-canonical DER signature"},
    {SCRIPT_ERR_MINIMALDATA, "MINIMALDATA", "Data push larger than necessary"},
    {SCRIPT_ERR_SIG_PUSHONLY, "SIG_PUSHONLY", "Only non-push operators allowed in signatures"},
    {SCRIPT_ERR_SIG_HIGH_S, "SIG_HIGH_S", "Non-canonical signature: S value is unnecessarily high"},
    {SCRIPT_ERR_SIG_NULLDUMMY, "SIG_NULLDUMMY", "Dummy CHECKMULTISIG argument must be zero"},
    {SCRIPT_ERR_PUBKEYTYPE, "PUBKEYTYPE", "Public key is neither compressed or uncompressed"},
    {SCRIPT_ERR_CLEANSTACK, "CLEANSTACK", "Extra items left on stack after execution"},
    {SCRIPT_ERR_MINIMALIF, "MINIMALIF", "OP_IF/NOTIF argument must be minimal"},
    {SCRIPT_ERR_SIG_NULLFAIL, "NULLFAIL", "Signature must be zero for failed CHECK(MULTI)SIG operation"},
    {SCRIPT_ERR_DISCOURAGE_UPGRADABLE_NOPS, "DISCOURAGE_UPGRADABLE_NOPS", "NOPx reserved for soft-fork upgrades"},
    {SCRIPT_ERR_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM, "DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM",
     "Witness version reserved for soft-fork upgrades"},
    {SCRIPT_ERR_NONCOMPRESSED_PUBKEY, "NONCOMPRESSED_PUBKEY", "Using non-compressed public key"},
    {SCRIPT_ERR_ILLEGAL_FORKID, "ILLEGAL_FORKID", "Illegal use of SIGHASH_FORKID"},
    {SCRIPT_ERR_MUST_USE_FORKID, "MISSING_FORKID", "Signature must use SIGHASH_FORKID"},
};

const std::pair<const char*, uint32_t> kFlagNames[] = {
    {"NONE", SCRIPT_VERIFY_NONE},
    {"P2SH", SCRIPT_VERIFY_P2SH},
    {"STRICTENC", SCRIPT_VERIFY_STRICTENC},
    {"DERSIG", SCRIPT_VERIFY_DERSIG},
    {"LOW_S", SCRIPT_VERIFY_LOW_S},
    {"SIGPUSHONLY", SCRIPT_VERIFY_SIGPUSHONLY},
    {"MINIMALDATA", SCRIPT_VERIFY_MINIMALDATA},
    {"NULLDUMMY", SCRIPT_VERIFY_NULLDUMMY},
    {"DISCOURAGE_UPGRADABLE_NOPS", SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS},
    {"CLEANSTACK", SCRIPT_VERIFY_CLEANSTACK},
    {"MINIMALIF", SCRIPT_VERIFY_MINIMALIF},
    {"NULLFAIL", SCRIPT_VERIFY_NULLFAIL},
    {"CHECKLOCKTIMEVERIFY", SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY},
    {"CHECKSEQUENCEVERIFY", SCRIPT_VERIFY_CHECKSEQUENCEVERIFY},
    {"DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM", SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM},
    {"COMPRESSED_PUBKEYTYPE", SCRIPT_VERIFY_COMPRESSED_PUBKEYTYPE},
    {"SIGHASH_FORKID", SCRIPT_ENABLE_SIGHASH_FORKID},
    {"ALLOW_NON_FORKID", SCRIPT_ALLOW_NON_FORKID},
};

inline bool set_success(ScriptError* ret) {
    if (ret) *ret = SCRIPT_ERR_OK;
    return true;
}
inline bool set_error(ScriptError* ret, ScriptError serror) {
    if (ret) *ret = serror;
    return false;
}
} // namespace

const char* ScriptErrorName(ScriptError err) {
    for (const auto& e : kErrors)
        if (e.e == err) return e.name;
    return "UNKNOWN_ERROR";
}
const char* ScriptErrorString(ScriptError err) {
    for (const auto& e : kErrors)
        if (e.e == err) return e.text;
    return "unknown error";
}
bool ParseScriptErrorName(const std::string& name, ScriptError& out) {
    for (const auto& e : kErrors)
        if (name == e.name) {
            out = e.e;
            return true;
        }
    return false;
}
uint32_t ParseScriptFlags(const std::string& s) {
    uint32_t flags = 0;
    if (s.empty()) return 0;
    size_t start = 0;
    while (start <= s.size()) {
        size_t comma = s.find(',', start);
        if (comma == std::string::npos) comma = s.size();
        const std::string w = s.substr(start, comma - start);
        bool found = false;
        for (const auto& f : kFlagNames)
            if (w == f.first) {
                flags |= f.second;
                found = true;
            }
        if (!found) throw std::invalid_argument("unknown script flag '" + w + "'");
        start = comma + 1;
    }
    return flags;
}
std::string FormatScriptFlags(uint32_t flags) {
    std::string r;
    for (const auto& f : kFlagNames)
        if (f.second && (flags & f.second)) r += std::string(r.empty() ? "" : ",") + f.first;
    return r;
}

// ------------------------------------------------------------------ helpers
bool CastToBool(const valtype& vch) {
    for (size_t i = 0; i < vch.size(); i++) {
        if (vch[i] != 0) {
            // negative zero is false
            if (i == vch.size() - 1 && vch[i] == 0x80) return false;
            return true;
        }
    }
    return false;
}

static inline valtype& stacktop(std::vector<valtype>& st, int i) { return st[st.size() + i]; }
static inline void popstack(std::vector<valtype>& st) {
    if (st.empty()) throw std::runtime_error("popstack(): stack empty");
    st.pop_back();
}

static bool IsCompressedOrUncompressedPubKey(const valtype& pk) {
    if (pk.size() < 33) return false;
    if (pk[0] == 0x04) return pk.size() == 65;
    if (pk[0] == 0x02 || pk[0] == 0x03) return pk.size() == 33;
    return false;
}
static bool IsCompressedPubKey(const valtype& pk) { return pk.size() == 33 && (pk[0] == 0x02 || pk[0] == 0x03); }

// BIP66 strict DER check over sig||hashtype.
bool IsValidSignatureEncoding(const valtype& sig) {
    if (sig.size() < 9 || sig.size() > 73) return false;
    if (sig[0] != 0x30) return false;
    if (sig[1] != sig.size() - 3) return false;
    const unsigned lenR = sig[3];
    if (5 + lenR >= sig.size()) return false;
    const unsigned lenS = sig[5 + lenR];
    if ((size_t)(lenR + lenS + 7) != sig.size()) return false;
    if (sig[2] != 0x02) return false;
    if (lenR == 0) return false;
    if (sig[4] & 0x80) return false;
    if (lenR > 1 && sig[4] == 0x00 && !(sig[5] & 0x80)) return false;
    if (sig[lenR + 4] != 0x02) return false;
    if (lenS == 0) return false;
    if (sig[lenR + 6] & 0x80) return false;
    if (lenS > 1 && sig[lenR + 6] == 0x00 && !(sig[lenR + 7] & 0x80)) return false;
    return true;
}

static uint32_t GetHashType(const valtype& sig) { return sig.empty() ? 0 : sig.back(); }

static bool IsLowDERSignature(const valtype& sig, ScriptError* serror) {
    if (!IsValidSignatureEncoding(sig)) return set_error(serror, SCRIPT_ERR_SIG_DER);
    valtype body(sig.begin(), sig.end() - 1);
    if (!CPubKey::CheckLowS(body)) return set_error(serror, SCRIPT_ERR_SIG_HIGH_S);
    return true;
}

static bool IsDefinedHashtypeSignature(const valtype& sig) {
    if (sig.empty()) return false;
    const uint32_t t = GetHashType(sig) & ~(uint32_t)(SIGHASH_ANYONECANPAY | SIGHASH_FORKID);
    return t >= SIGHASH_ALL && t <= SIGHASH_SINGLE;
}

bool CheckSignatureEncoding(const valtype& sig, uint32_t flags, ScriptError* serror) {
    if (sig.empty()) return true; // compact invalid signature for CHECK(MULTI)SIG
    if ((flags & (SCRIPT_VERIFY_DERSIG | SCRIPT_VERIFY_LOW_S | SCRIPT_VERIFY_STRICTENC)) != 0 &&
        !IsValidSignatureEncoding(sig))
        return set_error(serror, SCRIPT_ERR_SIG_DER);
    if ((flags & SCRIPT_VERIFY_LOW_S) != 0 && !IsLowDERSignature(sig, serror)) return false;
    if ((flags & SCRIPT_VERIFY_STRICTENC) != 0) {
        if (!IsDefinedHashtypeSignature(sig)) return set_error(serror, SCRIPT_ERR_SIG_HASHTYPE);
        const bool requires_forkid = !(flags & SCRIPT_ALLOW_NON_FORKID);
        const bool uses_forkid = (GetHashType(sig) & SIGHASH_FORKID) != 0;
        const bool forkid_enabled = (flags & SCRIPT_ENABLE_SIGHASH_FORKID) != 0;
        if (!forkid_enabled && uses_forkid && requires_forkid) return set_error(serror, SCRIPT_ERR_ILLEGAL_FORKID);
        if (forkid_enabled && !uses_forkid && requires_forkid) return set_error(serror, SCRIPT_ERR_MUST_USE_FORKID);
    }
    return true;
}

static bool CheckPubKeyEncoding(const valtype& pk, uint32_t flags, ScriptError* serror) {
    if ((flags & SCRIPT_VERIFY_STRICTENC) != 0 && !IsCompressedOrUncompressedPubKey(pk))
        return set_error(serror, SCRIPT_ERR_PUBKEYTYPE);
    if ((flags & SCRIPT_VERIFY_COMPRESSED_PUBKEYTYPE) && !IsCompressedPubKey(pk))
        return set_error(serror, SCRIPT_ERR_NONCOMPRESSED_PUBKEY);
    return true;
}

static bool CheckMinimalPush(const valtype& data, opcodetype opcode) {
    if (data.empty()) return opcode == OP_0;
    if (data.size() == 1 && data[0] >= 1 && data[0] <= 16) return opcode == OP_1 + (data[0] - 1);
    if (data.size() == 1 && data[0] == 0x81) return opcode == OP_1NEGATE;
    if (data.size() <= 75) return opcode == (int)data.size();
    if (data.size() <= 255) return opcode == OP_PUSHDATA1;
    if (data.size() <= 65535) return opcode == OP_PUSHDATA2;
    return true;
}

// Without FORKID the signature itself is removed from the scriptCode (legacy digest).
static void CleanupScriptCode(CScript& scriptCode, const valtype& sig, uint32_t flags) {
    const uint32_t ht = GetHashType(sig);
    if (!(flags & SCRIPT_ENABLE_SIGHASH_FORKID) || !(ht & SIGHASH_FORKID)) {
        CScript s;
        s << sig;
        scriptCode.FindAndDelete(s);
    }
}

static bool IsDisabledOpcode(opcodetype op) {
    switch (op) {
    case OP_CAT: case OP_SUBSTR: case OP_LEFT: case OP_RIGHT: case OP_INVERT: case OP_AND: case OP_OR:
    case OP_XOR: case OP_2MUL: case OP_2DIV: case OP_MUL: case OP_DIV: case OP_MOD: case OP_LSHIFT:
    case OP_RSHIFT:
        return true;
    default:
        return false;
    }
}

// ------------------------------------------------------------------ EvalScript
bool EvalScript(std::vector<valtype>& stack, const CScript& script, uint32_t flags,
                const BaseSignatureChecker& checker, ScriptError* serror) {
    static const CScriptNum bnZero(0);
    static const CScriptNum bnOne(1);
    static const valtype vchFalse(0);
    static const valtype vchTrue(1, 1);

    CScript::const_iterator pc = script.begin();
    const CScript::const_iterator pend = script.end();
    CScript::const_iterator pbegincodehash = script.begin();
    opcodetype opcode;
    valtype vchPushValue;
    std::vector<bool> vfExec;
    std::vector<valtype> altstack;
    set_error(serror, SCRIPT_ERR_UNKNOWN_ERROR);
    if (script.size() > (size_t)MAX_SCRIPT_SIZE) return set_error(serror, SCRIPT_ERR_SCRIPT_SIZE);
    int nOpCount = 0;
    const bool fRequireMinimal = (flags & SCRIPT_VERIFY_MINIMALDATA) != 0;
    const bool nullfail = (flags & SCRIPT_VERIFY_NULLFAIL) != 0;
    int nFalse = 0; // number of false entries in vfExec (O(1) fExec)

    try {
        while (pc < pend) {
            const bool fExec = nFalse == 0;
            if (!script.GetOp(pc, opcode, vchPushValue)) return set_error(serror, SCRIPT_ERR_BAD_OPCODE);
            if (vchPushValue.size() > MAX_SCRIPT_ELEMENT_SIZE) return set_error(serror, SCRIPT_ERR_PUSH_SIZE);
            if (opcode > OP_16 && ++nOpCount > MAX_OPS_PER_SCRIPT) return set_error(serror, SCRIPT_ERR_OP_COUNT);
            if (IsDisabledOpcode(opcode)) return set_error(serror, SCRIPT_ERR_DISABLED_OPCODE);

            if (fExec && 0 <= opcode && opcode <= OP_PUSHDATA4) {
                if (fRequireMinimal && !CheckMinimalPush(vchPushValue, opcode))
                    return set_error(serror, SCRIPT_ERR_MINIMALDATA);
                stack.push_back(vchPushValue);
            } else if (fExec || (OP_IF <= opcode && opcode <= OP_ENDIF)) {
                switch (opcode) {
                case OP_1NEGATE: case OP_1: case OP_2: case OP_3: case OP_4: case OP_5: case OP_6: case OP_7:
                case OP_8: case OP_9: case OP_10: case OP_11: case OP_12: case OP_13: case OP_14: case OP_15:
                case OP_16: {
                    CScriptNum bn((int)opcode - (int)(OP_1 - 1));
                    stack.push_back(bn.getvch());
                } break;

                case OP_NOP:
                    break;

                case OP_CHECKLOCKTIMEVERIFY: {
                    if (!(flags & SCRIPT_VERIFY_CHECKLOCKTIMEVERIFY)) {
                        if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS)
                            return set_error(serror, SCRIPT_ERR_DISCOURAGE_UPGRADABLE_NOPS);
                        break;
                    }
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    // 5-byte operands: nLockTime is uint32 (avoids a 2038 problem)
                    const CScriptNum nLockTime(stacktop(stack, -1), fRequireMinimal, 5);
                    if (nLockTime < 0) return set_error(serror, SCRIPT_ERR_NEGATIVE_LOCKTIME);
                    if (!checker.CheckLockTime(nLockTime)) return set_error(serror, SCRIPT_ERR_UNSATISFIED_LOCKTIME);
                } break;

                case OP_CHECKSEQUENCEVERIFY: {
                    if (!(flags & SCRIPT_VERIFY_CHECKSEQUENCEVERIFY)) {
                        if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS)
                            return set_error(serror, SCRIPT_ERR_DISCOURAGE_UPGRADABLE_NOPS);
                        break;
                    }
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    const CScriptNum nSequence(stacktop(stack, -1), fRequireMinimal, 5);
                    if (nSequence < 0) return set_error(serror, SCRIPT_ERR_NEGATIVE_LOCKTIME);
                    // disable flag set: behaves as a NOP
                    if ((nSequence & CTxIn::SEQUENCE_LOCKTIME_DISABLE_FLAG) != 0) break;
                    if (!checker.CheckSequence(nSequence)) return set_error(serror, SCRIPT_ERR_UNSATISFIED_LOCKTIME);
                } break;

                case OP_NOP1: case OP_NOP4: case OP_NOP5: case OP_NOP6: case OP_NOP7: case OP_NOP8: case OP_NOP9:
                case OP_NOP10:
                    if (flags & SCRIPT_VERIFY_DISCOURAGE_UPGRADABLE_NOPS)
                        return set_error(serror, SCRIPT_ERR_DISCOURAGE_UPGRADABLE_NOPS);
                    break;

                case OP_IF:
                case OP_NOTIF: {
                    bool fValue = false;
                    if (fExec) {
                        if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_UNBALANCED_CONDITIONAL);
                        valtype& vch = stacktop(stack, -1);
                        if (flags & SCRIPT_VERIFY_MINIMALIF) {
                            if (vch.size() > 1) return set_error(serror, SCRIPT_ERR_MINIMALIF);
                            if (vch.size() == 1 && vch[0] != 1) return set_error(serror, SCRIPT_ERR_MINIMALIF);
                        }
                        fValue = CastToBool(vch);
                        if (opcode == OP_NOTIF) fValue = !fValue;
                        popstack(stack);
                    }
                    vfExec.push_back(fValue);
                    if (!fValue) ++nFalse;
                } break;

                case OP_ELSE: {
                    if (vfExec.empty()) return set_error(serror, SCRIPT_ERR_UNBALANCED_CONDITIONAL);
                    nFalse += vfExec.back() ? 1 : -1;
                    vfExec.back() = !vfExec.back();
                } break;

                case OP_ENDIF: {
                    if (vfExec.empty()) return set_error(serror, SCRIPT_ERR_UNBALANCED_CONDITIONAL);
                    if (!vfExec.back()) --nFalse;
                    vfExec.pop_back();
                } break;

                case OP_VERIFY: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    if (CastToBool(stacktop(stack, -1))) popstack(stack);
                    else return set_error(serror, SCRIPT_ERR_VERIFY);
                } break;

                case OP_RETURN:
                    return set_error(serror, SCRIPT_ERR_OP_RETURN);

                // ---- stack ops
                case OP_TOALTSTACK: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    altstack.push_back(stacktop(stack, -1));
                    popstack(stack);
                } break;
                case OP_FROMALTSTACK: {
                    if (altstack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_ALTSTACK_OPERATION);
                    stack.push_back(altstack.back());
                    altstack.pop_back();
                } break;
                case OP_2DROP: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    popstack(stack);
                    popstack(stack);
                } break;
                case OP_2DUP: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype a = stacktop(stack, -2), b = stacktop(stack, -1);
                    stack.push_back(a);
                    stack.push_back(b);
                } break;
                case OP_3DUP: {
                    if (stack.size() < 3) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype a = stacktop(stack, -3), b = stacktop(stack, -2), c = stacktop(stack, -1);
                    stack.push_back(a);
                    stack.push_back(b);
                    stack.push_back(c);
                } break;
                case OP_2OVER: {
                    if (stack.size() < 4) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype a = stacktop(stack, -4), b = stacktop(stack, -3);
                    stack.push_back(a);
                    stack.push_back(b);
                } break;
                case OP_2ROT: {
                    if (stack.size() < 6) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype a = stacktop(stack, -6), b = stacktop(stack, -5);
                    stack.erase(stack.end() - 6, stack.end() - 4);
                    stack.push_back(a);
                    stack.push_back(b);
                } break;
                case OP_2SWAP: {
                    if (stack.size() < 4) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    std::swap(stacktop(stack, -4), stacktop(stack, -2));
                    std::swap(stacktop(stack, -3), stacktop(stack, -1));
                } break;
                case OP_IFDUP: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype v = stacktop(stack, -1);
                    if (CastToBool(v)) stack.push_back(v);
                } break;
                case OP_DEPTH: {
                    CScriptNum bn((int64_t)stack.size());
                    stack.push_back(bn.getvch());
                } break;
                case OP_DROP: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    popstack(stack);
                } break;
                case OP_DUP: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    stack.push_back(stacktop(stack, -1)); // push_back copies an aliased element safely
                } break;
                case OP_NIP: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    stack.erase(stack.end() - 2);
                } break;
                case OP_OVER: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype v = stacktop(stack, -2);
                    stack.push_back(v);
                } break;
                case OP_PICK:
                case OP_ROLL: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    const int n = CScriptNum(stacktop(stack, -1), fRequireMinimal).getint();
                    popstack(stack);
                    if (n < 0 || n >= (int)stack.size()) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype v = stacktop(stack, -n - 1);
                    if (opcode == OP_ROLL) stack.erase(stack.end() - n - 1);
                    stack.push_back(v);
                } break;
                case OP_ROT: {
                    if (stack.size() < 3) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    std::swap(stacktop(stack, -3), stacktop(stack, -2));
                    std::swap(stacktop(stack, -2), stacktop(stack, -1));
                } break;
                case OP_SWAP: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    std::swap(stacktop(stack, -2), stacktop(stack, -1));
                } break;
                case OP_TUCK: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype v = stacktop(stack, -1);
                    stack.insert(stack.end() - 2, v);
                } break;
                case OP_SIZE: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    CScriptNum bn((int64_t)stacktop(stack, -1).size());
                    stack.push_back(bn.getvch());
                } break;

                // ---- bitwise logic
                case OP_EQUAL:
                case OP_EQUALVERIFY: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    const bool fEqual = stacktop(stack, -2) == stacktop(stack, -1);
                    popstack(stack);
                    popstack(stack);
                    stack.push_back(fEqual ? vchTrue : vchFalse);
                    if (opcode == OP_EQUALVERIFY) {
                        if (fEqual) popstack(stack);
                        else return set_error(serror, SCRIPT_ERR_EQUALVERIFY);
                    }
                } break;

                // ---- numeric
                case OP_1ADD: case OP_1SUB: case OP_NEGATE: case OP_ABS: case OP_NOT: case OP_0NOTEQUAL: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    CScriptNum bn(stacktop(stack, -1), fRequireMinimal);
                    switch (opcode) {
                    case OP_1ADD: bn += 1; break;
                    case OP_1SUB: bn -= 1; break;
                    case OP_NEGATE: bn = -bn; break;
                    case OP_ABS: if (bn < bnZero) bn = -bn; break;
                    case OP_NOT: bn = CScriptNum(bn == bnZero); break;
                    case OP_0NOTEQUAL: bn = CScriptNum(bn != bnZero); break;
                    default: break;
                    }
                    popstack(stack);
                    stack.push_back(bn.getvch());
                } break;

                case OP_ADD: case OP_SUB: case OP_BOOLAND: case OP_BOOLOR: case OP_NUMEQUAL: case OP_NUMEQUALVERIFY:
                case OP_NUMNOTEQUAL: case OP_LESSTHAN: case OP_GREATERTHAN: case OP_LESSTHANOREQUAL:
                case OP_GREATERTHANOREQUAL: case OP_MIN: case OP_MAX: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    CScriptNum bn1(stacktop(stack, -2), fRequireMinimal);
                    CScriptNum bn2(stacktop(stack, -1), fRequireMinimal);
                    CScriptNum bn(0);
                    switch (opcode) {
                    case OP_ADD: bn = bn1 + bn2; break;
                    case OP_SUB: bn = bn1 - bn2; break;
                    case OP_BOOLAND: bn = CScriptNum(bn1 != bnZero && bn2 != bnZero); break;
                    case OP_BOOLOR: bn = CScriptNum(bn1 != bnZero || bn2 != bnZero); break;
                    case OP_NUMEQUAL: bn = CScriptNum(bn1 == bn2); break;
                    case OP_NUMEQUALVERIFY: bn = CScriptNum(bn1 == bn2); break;
                    case OP_NUMNOTEQUAL: bn = CScriptNum(bn1 != bn2); break;
                    case OP_LESSTHAN: bn = CScriptNum(bn1 < bn2); break;
                    case OP_GREATERTHAN: bn = CScriptNum(bn1 > bn2); break;
                    case OP_LESSTHANOREQUAL: bn = CScriptNum(bn1 <= bn2); break;
                    case OP_GREATERTHANOREQUAL: bn = CScriptNum(bn1 >= bn2); break;
                    case OP_MIN: bn = (bn1 < bn2 ? bn1 : bn2); break;
                    case OP_MAX: bn = (bn1 > bn2 ? bn1 : bn2); break;
                    default: break;
                    }
                    popstack(stack);
                    popstack(stack);
                    stack.push_back(bn.getvch());
                    if (opcode == OP_NUMEQUALVERIFY) {
                        if (CastToBool(stacktop(stack, -1))) popstack(stack);
                        else return set_error(serror, SCRIPT_ERR_NUMEQUALVERIFY);
                    }
                } break;

                case OP_WITHIN: {
                    if (stack.size() < 3) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    CScriptNum bn1(stacktop(stack, -3), fRequireMinimal);
                    CScriptNum bn2(stacktop(stack, -2), fRequireMinimal);
                    CScriptNum bn3(stacktop(stack, -1), fRequireMinimal);
                    const bool fValue = (bn2 <= bn1 && bn1 < bn3);
                    popstack(stack);
                    popstack(stack);
                    popstack(stack);
                    stack.push_back(fValue ? vchTrue : vchFalse);
                } break;

                // ---- crypto
                case OP_RIPEMD160: case OP_SHA1: case OP_SHA256: case OP_HASH160: case OP_HASH256: {
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype& vch = stacktop(stack, -1);
                    valtype vchHash((opcode == OP_RIPEMD160 || opcode == OP_SHA1 || opcode == OP_HASH160) ? 20 : 32);
                    if (opcode == OP_RIPEMD160) CRIPEMD160().Write(vch.data(), vch.size()).Finalize(vchHash.data());
                    else if (opcode == OP_SHA1) CSHA1().Write(vch.data(), vch.size()).Finalize(vchHash.data());
                    else if (opcode == OP_SHA256) CSHA256().Write(vch.data(), vch.size()).Finalize(vchHash.data());
                    else if (opcode == OP_HASH160) Hash160(vch.data(), vch.size(), vchHash.data());
                    else Sha256d(vch.data(), vch.size(), vchHash.data());
                    vch.swap(vchHash); // the digest replaces the top element in place
                } break;

                case OP_CODESEPARATOR:
                    pbegincodehash = pc;
                    break;

                case OP_CHECKSIG:
                case OP_CHECKSIGVERIFY: {
                    if (stack.size() < 2) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    valtype& vchSig = stacktop(stack, -2);
                    valtype& vchPubKey = stacktop(stack, -1);
                    CScript scriptCode(pbegincodehash, pend);
                    CleanupScriptCode(scriptCode, vchSig, flags);
                    if (!CheckSignatureEncoding(vchSig, flags, serror) || !CheckPubKeyEncoding(vchPubKey, flags, serror))
                        return false;
                    const bool deferrable = nullfail && !vchSig.empty();
                    const bool fSuccess = checker.CheckSig(vchSig, vchPubKey, scriptCode, flags, deferrable);
                    if (!fSuccess && nullfail && !vchSig.empty()) return set_error(serror, SCRIPT_ERR_SIG_NULLFAIL);
                    popstack(stack);
                    popstack(stack);
                    stack.push_back(fSuccess ? vchTrue : vchFalse);
                    if (opcode == OP_CHECKSIGVERIFY) {
                        if (fSuccess) popstack(stack);
                        else return set_error(serror, SCRIPT_ERR_CHECKSIGVERIFY);
                    }
                } break;

                case OP_CHECKMULTISIG:
                case OP_CHECKMULTISIGVERIFY: {
                    // ([sig ...] num_of_signatures [pubkey ...] num_of_pubkeys -- bool)
                    int i = 1;
                    if ((int)stack.size() < i) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    int nKeysCount = CScriptNum(stacktop(stack, -i), fRequireMinimal).getint();
                    if (nKeysCount < 0 || nKeysCount > MAX_PUBKEYS_PER_MULTISIG)
                        return set_error(serror, SCRIPT_ERR_PUBKEY_COUNT);
                    nOpCount += nKeysCount;
                    if (nOpCount > MAX_OPS_PER_SCRIPT) return set_error(serror, SCRIPT_ERR_OP_COUNT);
                    int ikey = ++i;
                    // ikey2 is the position of the last non-signature item in the stack
                    int ikey2 = nKeysCount + 2;
                    i += nKeysCount;
                    if ((int)stack.size() < i) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    int nSigsCount = CScriptNum(stacktop(stack, -i), fRequireMinimal).getint();
                    if (nSigsCount < 0 || nSigsCount > nKeysCount) return set_error(serror, SCRIPT_ERR_SIG_COUNT);
                    int isig = ++i;
                    i += nSigsCount;
                    if ((int)stack.size() < i) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);

                    CScript scriptCode(pbegincodehash, pend);
                    for (int k = 0; k < nSigsCount; k++) CleanupScriptCode(scriptCode, stacktop(stack, -isig - k), flags);

                    bool fSuccess = true;
                    // Speculative deferral (NULLFAIL, every signature non-empty and well encoded): a
                    // failed match would fail the script, so a batching checker may take the match
                    // over. It queues every (signature, key) pair the greedy match could try,
                    // m*(n-m+1) of them, where the eager loop verifies at most n (what sigop
                    // accounting charges): deferral is taken only while that is within 2n (1-of-n,
                    // n-of-n, 2-of-3, 3-of-5, ...), so a block of 10-of-20 spends at the sigop limit
                    // never costs more than twice the reference's worst case, on the GPU or on the CPU
                    // fallback. Otherwise the greedy loop below runs eagerly, as in the reference.
                    bool deferred = false;
                    if (nullfail && nSigsCount > 0 && nSigsCount * (nKeysCount - nSigsCount + 1) <= 2 * nKeysCount) {
                        std::vector<const valtype*> sigs, keys;
                        bool defer = true;
                        for (int k = 0; k < nSigsCount && defer; k++) {
                            const valtype& vs = stacktop(stack, -isig - k);
                            ScriptError e;
                            defer = !vs.empty() && CheckSignatureEncoding(vs, flags, &e);
                            sigs.push_back(&vs);
                        }
                        if (defer) {
                            uint32_t keyOk = 0;
                            for (int k = 0; k < nKeysCount; k++) {
                                const valtype& vk = stacktop(stack, -ikey - k);
                                ScriptError e;
                                if (CheckPubKeyEncoding(vk, flags, &e)) keyOk |= 1u << k;
                                keys.push_back(&vk);
                            }
                            deferred = checker.DeferMultisig(sigs, keys, keyOk, scriptCode, flags);
                        }
                    }
                    while (!deferred && fSuccess && nSigsCount > 0) {
                        valtype& vchSig = stacktop(stack, -isig);
                        valtype& vchPubKey = stacktop(stack, -ikey);
                        if (!CheckSignatureEncoding(vchSig, flags, serror) ||
                            !CheckPubKeyEncoding(vchPubKey, flags, serror))
                            return false;
                        // never deferred: a mismatching (sig, key) pair is legal here
                        const bool fOk = checker.CheckSig(vchSig, vchPubKey, scriptCode, flags, false);
                        if (fOk) {
                            isig++;
                            nSigsCount--;
                        }
                        ikey++;
                        nKeysCount--;
                        if (nSigsCount > nKeysCount) fSuccess = false;
                    }

                    // Clean up stack of actual arguments
                    while (i-- > 1) {
                        // NULLFAIL: all signatures must be empty if the check failed
                        if (!fSuccess && nullfail && !ikey2 && stacktop(stack, -1).size())
                            return set_error(serror, SCRIPT_ERR_SIG_NULLFAIL);
                        if (ikey2 > 0) ikey2--;
                        popstack(stack);
                    }
                    // Extra element (historical off-by-one): must be empty under NULLDUMMY
                    if (stack.size() < 1) return set_error(serror, SCRIPT_ERR_INVALID_STACK_OPERATION);
                    if ((flags & SCRIPT_VERIFY_NULLDUMMY) && stacktop(stack, -1).size())
                        return set_error(serror, SCRIPT_ERR_SIG_NULLDUMMY);
                    popstack(stack);
                    stack.push_back(fSuccess ? vchTrue : vchFalse);
                    if (opcode == OP_CHECKMULTISIGVERIFY) {
                        if (fSuccess) popstack(stack);
                        else return set_error(serror, SCRIPT_ERR_CHECKMULTISIGVERIFY);
                    }
                } break;

                default:
                    return set_error(serror, SCRIPT_ERR_BAD_OPCODE);
                }
            }

            if (stack.size() + altstack.size() > 1000) return set_error(serror, SCRIPT_ERR_STACK_SIZE);
        }
    } catch (...) {
        return set_error(serror, SCRIPT_ERR_UNKNOWN_ERROR);
    }

    if (!vfExec.empty()) return set_error(serror, SCRIPT_ERR_UNBALANCED_CONDITIONAL);
    return set_success(serror);
}

// ------------------------------------------------------------------ signature hash
namespace {
// Legacy (pre-FORKID) digest serializer (CTransactionSignatureSerializer semantics).
class LegacySigSerializer {
public:
    LegacySigSerializer(const CTransaction& tx, const CScript& code, unsigned nIn, uint32_t ht)
        : tx(tx), code(code), nIn(nIn), anyone(ht & SIGHASH_ANYONECANPAY), single((ht & 0x1f) == SIGHASH_SINGLE),
          none((ht & 0x1f) == SIGHASH_NONE) {}
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, tx.nVersion);
        const unsigned nInputs = anyone ? 1 : (unsigned)tx.vin.size();
        WriteCompactSize(s, nInputs);
        for (unsigned i = 0; i < nInputs; i++) SerializeInput(s, anyone ? nIn : i);
        const unsigned nOutputs = none ? 0 : (single ? nIn + 1 : (unsigned)tx.vout.size());
        WriteCompactSize(s, nOutputs);
        for (unsigned o = 0; o < nOutputs; o++) {
            if (single && o != nIn) ::bcp::Serialize(s, CTxOut());
            else ::bcp::Serialize(s, tx.vout[o]);
        }
        ::bcp::Serialize(s, tx.nLockTime);
    }

private:
    template <typename S> void SerializeScriptCode(S& s) const {
        // scriptCode with OP_CODESEPARATORs removed
        CScript::const_iterator it = code.begin(), itBegin = it;
        opcodetype op;
        unsigned nSeps = 0;
        while (code.GetOp(it, op))
            if (op == OP_CODESEPARATOR) nSeps++;
        WriteCompactSize(s, code.size() - nSeps);
        it = itBegin;
        while (code.GetOp(it, op)) {
            if (op == OP_CODESEPARATOR) {
                s.write((const char*)&itBegin[0], it - itBegin - 1);
                itBegin = it;
            }
        }
        if (itBegin != code.end()) s.write((const char*)&itBegin[0], it - itBegin);
    }
    template <typename S> void SerializeInput(S& s, unsigned nInput) const {
        ::bcp::Serialize(s, tx.vin[nInput].prevout);
        if (nInput != nIn) ::bcp::Serialize(s, CScript());
        else SerializeScriptCode(s);
        if (nInput != nIn && (single || none)) ::bcp::Serialize(s, (uint32_t)0);
        else ::bcp::Serialize(s, tx.vin[nInput].nSequence);
    }
    const CTransaction& tx;
    const CScript& code;
    const unsigned nIn;
    const bool anyone, single, none;
};

uint256 PrevoutsHash(const CTransaction& tx) {
    HashWriter ss;
    for (const auto& in : tx.vin) ss << in.prevout;
    return ss.GetHash();
}
uint256 SequenceHash(const CTransaction& tx) {
    HashWriter ss;
    for (const auto& in : tx.vin) ss << in.nSequence;
    return ss.GetHash();
}
uint256 OutputsHash(const CTransaction& tx) {
    HashWriter ss;
    for (const auto& out : tx.vout) ss << out;
    return ss.GetHash();
}
} // namespace

uint256 SignatureHash(const CScript& scriptCode, const CTransaction& txTo, unsigned int nIn, uint32_t nHashType,
                      Amount amount, const PrecomputedTransactionData* cache, uint32_t flags) {
    if ((nHashType & SIGHASH_FORKID) && (flags & SCRIPT_ENABLE_SIGHASH_FORKID)) {
        uint256 hashPrevouts, hashSequence, hashOutputs;
        const uint32_t base = nHashType & 0x1f;
        if (!(nHashType & SIGHASH_ANYONECANPAY)) hashPrevouts = cache ? cache->hashPrevouts : PrevoutsHash(txTo);
        if (!(nHashType & SIGHASH_ANYONECANPAY) && base != SIGHASH_SINGLE && base != SIGHASH_NONE)
            hashSequence = cache ? cache->hashSequence : SequenceHash(txTo);
        if (base != SIGHASH_SINGLE && base != SIGHASH_NONE) {
            hashOutputs = cache ? cache->hashOutputs : OutputsHash(txTo);
        } else if (base == SIGHASH_SINGLE && nIn < txTo.vout.size()) {
            HashWriter ss;
            ss << txTo.vout[nIn];
            hashOutputs = ss.GetHash();
        }
        HashWriter ss;
        ss << txTo.nVersion << hashPrevouts << hashSequence << txTo.vin[nIn].prevout
           << static_cast<const CScriptBase&>(scriptCode) << amount << txTo.vin[nIn].nSequence
           << hashOutputs << txTo.nLockTime << nHashType;
        return ss.GetHash();
    }
    static const uint256 one = uint256S("0000000000000000000000000000000000000000000000000000000000000001");
    if (nIn >= txTo.vin.size()) return one;
    if ((nHashType & 0x1f) == SIGHASH_SINGLE && nIn >= txTo.vout.size()) return one;
    HashWriter ss;
    ss << LegacySigSerializer(txTo, scriptCode, nIn, nHashType) << nHashType;
    return ss.GetHash();
}

// ------------------------------------------------------------------ checkers
bool TransactionSignatureChecker::PrepareSig(const valtype& sigIn, const CScript& scriptCode, uint32_t flags,
                                             valtype& sigOut, uint256& sighash) const {
    if (!SigDigest(sigIn, scriptCode, flags, sighash)) return false;
    sigOut.assign(sigIn.begin(), sigIn.end() - 1);
    return true;
}

bool TransactionSignatureChecker::SigDigest(const valtype& sigIn, const CScript& scriptCode, uint32_t flags,
                                            uint256& sighash) const {
    if (sigIn.empty()) return false;
    const uint32_t ht = sigIn.back();
    if (memoValid && ht == memoHashType && flags == memoFlags && scriptCode == memoCode) {
        sighash = memoSighash;
        return true;
    }
    sighash = SignatureHash(scriptCode, *txTo, nIn, ht, amount, txdata, flags);
    memoCode = scriptCode;
    memoHashType = ht;
    memoFlags = flags;
    memoSighash = sighash;
    memoValid = true;
    return true;
}

bool TransactionSignatureChecker::VerifySignature(const valtype& sig, const valtype& pubkey,
                                                  const uint256& sighash) const {
    return secp::VerifySignature(pubkey.data(), pubkey.size(), sig.data(), sig.size(), sighash.begin());
}

bool TransactionSignatureChecker::CheckSig(const valtype& sigIn, const valtype& pubkey, const CScript& scriptCode,
                                           uint32_t flags, bool) const {
    if (CPubKey::GetLen(pubkey.empty() ? 0 : pubkey[0]) != pubkey.size() || pubkey.empty()) return false;
    valtype sig;
    uint256 sighash;
    if (!PrepareSig(sigIn, scriptCode, flags, sig, sighash)) return false;
    return VerifySignature(sig, pubkey, sighash);
}

bool DeferringSignatureChecker::CheckSig(const valtype& sigIn, const valtype& pubkey, const CScript& scriptCode,
                                         uint32_t flags, bool deferrable) const {
    if (!deferrable || !sink) return TransactionSignatureChecker::CheckSig(sigIn, pubkey, scriptCode, flags, false);
    if (pubkey.empty() || CPubKey::GetLen(pubkey[0]) != pubkey.size()) return false;
    // a signature or key too long for the inline record (only possible without STRICTENC) is
    // checked right away
    if (sigIn.empty()) return false;
    if (sigIn.size() - 1 > decltype(DeferredSigCheck::sig)::capacity ||
        pubkey.size() > decltype(DeferredSigCheck::pubkey)::capacity)
        return TransactionSignatureChecker::CheckSig(sigIn, pubkey, scriptCode, flags, false);
    sink->emplace_back();
    DeferredSigCheck& c = sink->back();
    if (!SigDigest(sigIn, scriptCode, flags, c.sighash)) {
        sink->pop_back();
        return false;
    }
    c.sig.assign(sigIn.data(), sigIn.size() - 1);
    c.pubkey.assign(pubkey);
    return true;
}

bool DeferringSignatureChecker::DeferMultisig(const std::vector<const valtype*>& sigs,
                                              const std::vector<const valtype*>& keys, uint32_t keyOk,
                                              const CScript& scriptCode, uint32_t flags) const {
    if (!sink || !groups) return false;
    const size_t m = sigs.size(), n = keys.size();
    if (m == 0 || m > n || n > MAX_PUBKEYS_PER_MULTISIG) return false;
    for (const valtype* k : keys)
        if (k->size() > decltype(DeferredSigCheck::pubkey)::capacity) return false;
    std::vector<uint256> digests(m);
    for (size_t i = 0; i < m; i++) {
        if (sigs[i]->empty() || sigs[i]->size() - 1 > decltype(DeferredSigCheck::sig)::capacity) return false;
        if (!SigDigest(*sigs[i], scriptCode, flags, digests[i])) return false;
    }
    DeferredMultisig g;
    g.first = (uint32_t)sink->size();
    g.m = (uint8_t)m;
    g.n = (uint8_t)n;
    g.keyOk = keyOk;
    sink->reserve(sink->size() + g.Pairs());
    for (size_t i = 0; i < m; i++) {
        for (size_t j = i; j <= i + (n - m); j++) {
            sink->emplace_back();
            DeferredSigCheck& c = sink->back();
            c.sighash = digests[i];
            c.sig.assign(sigs[i]->data(), sigs[i]->size() - 1);
            const valtype& k = *keys[j];
            // a key that would fail parsing verifies as false, as the eager check would
            if (!k.empty() && CPubKey::GetLen(k[0]) == k.size()) c.pubkey.assign(k);
        }
    }
    groups->push_back(g);
    return true;
}

bool EvalDeferredMultisig(const DeferredMultisig& g, const uint8_t* pairResults) {
    const int m = g.m, n = g.n, width = n - m + 1;
    int isig = 0, ikey = 0, nSigs = m, nKeys = n;
    bool fSuccess = true;
    while (fSuccess && nSigs > 0) {
        if (!((g.keyOk >> ikey) & 1)) return false; // a visited key that fails encoding: script error
        // (while matching, 0 <= ikey - isig <= n - m: the pair is one of the recorded ones)
        if (pairResults[isig * width + (ikey - isig)]) {
            isig++;
            nSigs--;
        }
        ikey++;
        nKeys--;
        if (nSigs > nKeys) fSuccess = false;
    }
    return fSuccess;
}

bool TransactionSignatureChecker::CheckLockTime(const CScriptNum& nLockTime) const {
    // same kind (height vs time) on both sides
    if (!((txTo->nLockTime < LOCKTIME_THRESHOLD && nLockTime < LOCKTIME_THRESHOLD) ||
          (txTo->nLockTime >= LOCKTIME_THRESHOLD && nLockTime >= LOCKTIME_THRESHOLD)))
        return false;
    if (nLockTime > (int64_t)txTo->nLockTime) return false;
    // a final input would bypass nLockTime entirely
    if (CTxIn::SEQUENCE_FINAL == txTo->vin[nIn].nSequence) return false;
    return true;
}

bool TransactionSignatureChecker::CheckSequence(const CScriptNum& nSequence) const {
    const int64_t txToSequence = (int64_t)txTo->vin[nIn].nSequence;
    if ((uint32_t)txTo->nVersion < 2) return false;
    if (txToSequence & CTxIn::SEQUENCE_LOCKTIME_DISABLE_FLAG) return false;
    const uint32_t mask = CTxIn::SEQUENCE_LOCKTIME_TYPE_FLAG | CTxIn::SEQUENCE_LOCKTIME_MASK;
    const int64_t txSeqMasked = txToSequence & mask;
    const CScriptNum seqMasked = nSequence & mask;
    if (!((txSeqMasked < CTxIn::SEQUENCE_LOCKTIME_TYPE_FLAG && seqMasked < CTxIn::SEQUENCE_LOCKTIME_TYPE_FLAG) ||
          (txSeqMasked >= CTxIn::SEQUENCE_LOCKTIME_TYPE_FLAG && seqMasked >= CTxIn::SEQUENCE_LOCKTIME_TYPE_FLAG)))
        return false;
    if (seqMasked > txSeqMasked) return false;
    return true;
}

// ------------------------------------------------------------------ VerifyScript
bool VerifyScript(const CScript& scriptSig, const CScript& scriptPubKey, uint32_t flags,
                  const BaseSignatureChecker& checker, ScriptError* serror) {
    set_error(serror, SCRIPT_ERR_UNKNOWN_ERROR);
    if (flags & SCRIPT_ENABLE_SIGHASH_FORKID) flags |= SCRIPT_VERIFY_STRICTENC;
    if ((flags & SCRIPT_VERIFY_SIGPUSHONLY) != 0 && !scriptSig.IsPushOnly())
        return set_error(serror, SCRIPT_ERR_SIG_PUSHONLY);

    std::vector<valtype> stack, stackCopy;
    stack.reserve(8); // P2PKH / multisig / P2SH spends stay within it: no regrowth while evaluating
    if (!EvalScript(stack, scriptSig, flags, checker, serror)) return false;
    // the copy is only read for a P2SH output (below); the reference copies for every output
    const bool p2sh = (flags & SCRIPT_VERIFY_P2SH) && scriptPubKey.IsPayToScriptHash();
    if (p2sh) stackCopy = stack;
    if (!EvalScript(stack, scriptPubKey, flags, checker, serror)) return false;
    if (stack.empty() || !CastToBool(stack.back())) return set_error(serror, SCRIPT_ERR_EVAL_FALSE);

    if (p2sh) {
        if (!scriptSig.IsPushOnly()) return set_error(serror, SCRIPT_ERR_SIG_PUSHONLY);
        std::swap(stack, stackCopy);
        // non-empty: HASH160 <h> EQUAL over an empty stack would have failed above
        const valtype redeem = stack.back();
        CScript pubKey2(redeem.begin(), redeem.end());
        popstack(stack);
        if (!EvalScript(stack, pubKey2, flags, checker, serror)) return false;
        if (stack.empty() || !CastToBool(stack.back())) return set_error(serror, SCRIPT_ERR_EVAL_FALSE);
    }

    if ((flags & SCRIPT_VERIFY_CLEANSTACK) != 0) {
        if (!(flags & SCRIPT_VERIFY_P2SH)) throw std::logic_error("CLEANSTACK requires P2SH");
        if (stack.size() != 1) return set_error(serror, SCRIPT_ERR_CLEANSTACK);
    }
    return set_success(serror);
}

} // namespace bcp
