// Script container, opcodes and script number arithmetic.
// Behaviour parity: reference src/script/script.{h,cpp} (opcodetype, CScriptNum with
// minimal-encoding checks, CScript::GetOp, GetSigOpCount, IsPayToScriptHash,
// IsPushOnly, IsUnspendable, IsCommitment for the BCP anti-replay OP_RETURN
// (script.cpp:316-333)).
#pragma once
#include "util/prevector.h"
#include "primitives/serialize.h"

#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace bcp {

static const unsigned int MAX_SCRIPT_ELEMENT_SIZE = 520;
static const int MAX_OPS_PER_SCRIPT = 201;
static const int MAX_PUBKEYS_PER_MULTISIG = 20;
static const int MAX_SCRIPT_SIZE = 10000;
static const unsigned int LOCKTIME_THRESHOLD = 500000000; // Tue Nov  5 00:53:20 1985 UTC

enum opcodetype {
    OP_0 = 0x00, OP_FALSE = OP_0, OP_PUSHDATA1 = 0x4c, OP_PUSHDATA2 = 0x4d, OP_PUSHDATA4 = 0x4e,
    OP_1NEGATE = 0x4f, OP_RESERVED = 0x50, OP_1 = 0x51, OP_TRUE = OP_1, OP_2 = 0x52, OP_3 = 0x53,
    OP_4 = 0x54, OP_5 = 0x55, OP_6 = 0x56, OP_7 = 0x57, OP_8 = 0x58, OP_9 = 0x59, OP_10 = 0x5a,
    OP_11 = 0x5b, OP_12 = 0x5c, OP_13 = 0x5d, OP_14 = 0x5e, OP_15 = 0x5f, OP_16 = 0x60,
    OP_NOP = 0x61, OP_VER = 0x62, OP_IF = 0x63, OP_NOTIF = 0x64, OP_VERIF = 0x65, OP_VERNOTIF = 0x66,
    OP_ELSE = 0x67, OP_ENDIF = 0x68, OP_VERIFY = 0x69, OP_RETURN = 0x6a,
    OP_TOALTSTACK = 0x6b, OP_FROMALTSTACK = 0x6c, OP_2DROP = 0x6d, OP_2DUP = 0x6e, OP_3DUP = 0x6f,
    OP_2OVER = 0x70, OP_2ROT = 0x71, OP_2SWAP = 0x72, OP_IFDUP = 0x73, OP_DEPTH = 0x74, OP_DROP = 0x75,
    OP_DUP = 0x76, OP_NIP = 0x77, OP_OVER = 0x78, OP_PICK = 0x79, OP_ROLL = 0x7a, OP_ROT = 0x7b,
    OP_SWAP = 0x7c, OP_TUCK = 0x7d,
    OP_CAT = 0x7e, OP_SUBSTR = 0x7f, OP_LEFT = 0x80, OP_RIGHT = 0x81, OP_SIZE = 0x82,
    OP_INVERT = 0x83, OP_AND = 0x84, OP_OR = 0x85, OP_XOR = 0x86, OP_EQUAL = 0x87, OP_EQUALVERIFY = 0x88,
    OP_RESERVED1 = 0x89, OP_RESERVED2 = 0x8a,
    OP_1ADD = 0x8b, OP_1SUB = 0x8c, OP_2MUL = 0x8d, OP_2DIV = 0x8e, OP_NEGATE = 0x8f, OP_ABS = 0x90,
    OP_NOT = 0x91, OP_0NOTEQUAL = 0x92, OP_ADD = 0x93, OP_SUB = 0x94, OP_MUL = 0x95, OP_DIV = 0x96,
    OP_MOD = 0x97, OP_LSHIFT = 0x98, OP_RSHIFT = 0x99, OP_BOOLAND = 0x9a, OP_BOOLOR = 0x9b,
    OP_NUMEQUAL = 0x9c, OP_NUMEQUALVERIFY = 0x9d, OP_NUMNOTEQUAL = 0x9e, OP_LESSTHAN = 0x9f,
    OP_GREATERTHAN = 0xa0, OP_LESSTHANOREQUAL = 0xa1, OP_GREATERTHANOREQUAL = 0xa2, OP_MIN = 0xa3,
    OP_MAX = 0xa4, OP_WITHIN = 0xa5,
    OP_RIPEMD160 = 0xa6, OP_SHA1 = 0xa7, OP_SHA256 = 0xa8, OP_HASH160 = 0xa9, OP_HASH256 = 0xaa,
    OP_CODESEPARATOR = 0xab, OP_CHECKSIG = 0xac, OP_CHECKSIGVERIFY = 0xad, OP_CHECKMULTISIG = 0xae,
    OP_CHECKMULTISIGVERIFY = 0xaf,
    OP_NOP1 = 0xb0, OP_CHECKLOCKTIMEVERIFY = 0xb1, OP_NOP2 = OP_CHECKLOCKTIMEVERIFY,
    OP_CHECKSEQUENCEVERIFY = 0xb2, OP_NOP3 = OP_CHECKSEQUENCEVERIFY, OP_NOP4 = 0xb3, OP_NOP5 = 0xb4,
    OP_NOP6 = 0xb5, OP_NOP7 = 0xb6, OP_NOP8 = 0xb7, OP_NOP9 = 0xb8, OP_NOP10 = 0xb9,
    OP_SMALLINTEGER = 0xfa, OP_PUBKEYS = 0xfb, OP_PUBKEYHASH = 0xfd, OP_PUBKEY = 0xfe,
    OP_INVALIDOPCODE = 0xff,
};

const char* GetOpName(opcodetype opcode);

class scriptnum_error : public std::runtime_error {
public:
    explicit scriptnum_error(const std::string& s) : std::runtime_error(s) {}
};

// Numeric stack values: little-endian sign-magnitude, max 4 bytes as operands.
class CScriptNum {
public:
    static const size_t MAXIMUM_ELEMENT_SIZE = 4;
    explicit CScriptNum(const int64_t& n) : m_value(n) {}
    explicit CScriptNum(const std::vector<unsigned char>& vch, bool fRequireMinimal,
                        const size_t nMaxNumSize = MAXIMUM_ELEMENT_SIZE);
    static bool IsMinimallyEncoded(const std::vector<unsigned char>& vch, size_t maxSize = MAXIMUM_ELEMENT_SIZE);

    bool operator==(const int64_t& rhs) const { return m_value == rhs; }
    bool operator!=(const int64_t& rhs) const { return m_value != rhs; }
    bool operator<=(const int64_t& rhs) const { return m_value <= rhs; }
    bool operator<(const int64_t& rhs) const { return m_value < rhs; }
    bool operator>=(const int64_t& rhs) const { return m_value >= rhs; }
    bool operator>(const int64_t& rhs) const { return m_value > rhs; }
    bool operator==(const CScriptNum& r) const { return m_value == r.m_value; }
    bool operator<(const CScriptNum& r) const { return m_value < r.m_value; }
    bool operator<=(const CScriptNum& r) const { return m_value <= r.m_value; }
    bool operator>(const CScriptNum& r) const { return m_value > r.m_value; }
    bool operator>=(const CScriptNum& r) const { return m_value >= r.m_value; }
    bool operator!=(const CScriptNum& r) const { return m_value != r.m_value; }
    CScriptNum operator+(const int64_t& r) const { return CScriptNum(m_value + r); }
    CScriptNum operator-(const int64_t& r) const { return CScriptNum(m_value - r); }
    CScriptNum operator+(const CScriptNum& r) const { return CScriptNum(m_value + r.m_value); }
    CScriptNum operator-(const CScriptNum& r) const { return CScriptNum(m_value - r.m_value); }
    CScriptNum operator-() const { return CScriptNum(-m_value); }
    CScriptNum& operator+=(const int64_t& r) { m_value += r; return *this; }
    CScriptNum& operator-=(const int64_t& r) { m_value -= r; return *this; }
    CScriptNum operator&(const int64_t& r) const { return CScriptNum(m_value & r); }

    int getint() const {
        if (m_value > std::numeric_limits<int>::max()) return std::numeric_limits<int>::max();
        if (m_value < std::numeric_limits<int>::min()) return std::numeric_limits<int>::min();
        return (int)m_value;
    }
    int64_t getint64() const { return m_value; }
    std::vector<unsigned char> getvch() const { return serialize(m_value); }
    static std::vector<unsigned char> serialize(const int64_t& value);

private:
    int64_t m_value;
};

// Script bytes: inline up to 28 (every standard output script), on the heap beyond
// (reference src/script/script.h:371 CScriptBase = prevector<28, unsigned char>)
typedef prevector<28, unsigned char> CScriptBase;

class CScript : public CScriptBase {
public:
    CScript() {}
    CScript(const_iterator b, const_iterator e) : CScriptBase(b, e) {}
    CScript(std::vector<unsigned char>::const_iterator b, std::vector<unsigned char>::const_iterator e) : CScriptBase(b, e) {}
    explicit CScript(const std::vector<unsigned char>& v) : CScriptBase(v.begin(), v.end()) {}
    explicit CScript(opcodetype op) { *this << op; }

    static opcodetype EncodeOP_N(int n) { return n == 0 ? OP_0 : (opcodetype)(OP_1 + n - 1); }
    static int DecodeOP_N(opcodetype op) { return op == OP_0 ? 0 : (int)op - (int)(OP_1 - 1); }

    CScript& operator<<(int64_t b) {
        if (b == -1 || (b >= 1 && b <= 16)) push_back((unsigned char)(b + (OP_1 - 1)));
        else if (b == 0) push_back(OP_0);
        else *this << CScriptNum::serialize(b);
        return *this;
    }
    CScript& operator<<(opcodetype op) {
        if (op < 0 || op > 0xff) throw std::runtime_error("CScript::operator<<(): invalid opcode");
        insert(end(), (unsigned char)op);
        return *this;
    }
    CScript& operator<<(const CScriptNum& b) { *this << b.getvch(); return *this; }
    CScript& operator<<(const std::vector<unsigned char>& b);
    CScript& operator<<(const CScript&) = delete;

    bool GetOp(const_iterator& pc, opcodetype& opcodeRet, std::vector<unsigned char>& vchRet) const;
    bool GetOp(const_iterator& pc, opcodetype& opcodeRet) const;

    unsigned int GetSigOpCount(bool fAccurate) const;
    unsigned int GetSigOpCount(const CScript& scriptSig) const; // P2SH-aware
    bool IsPayToScriptHash() const;
    bool IsPushOnly(const_iterator pc) const;
    bool IsPushOnly() const { return IsPushOnly(begin()); }
    // OP_RETURN <push of exactly `commitment`> (reference script.cpp:316-333).
    bool IsCommitment(const std::vector<unsigned char>& commitment) const;
    bool IsUnspendable() const { return (size() > 0 && *begin() == OP_RETURN) || (size() > MAX_SCRIPT_SIZE); }
    void clear() { CScriptBase::clear(); }
    std::string ToString() const;
    // Remove all occurrences of a serialized sub-script (legacy FindAndDelete).
    int FindAndDelete(const CScript& b);

    template <typename S> void Serialize(S& s) const { ::bcp::Serialize(s, static_cast<const CScriptBase&>(*this)); }
    template <typename S> void Unserialize(S& s) { ::bcp::Unserialize(s, static_cast<CScriptBase&>(*this)); }
};

// Parse a script from the human-readable assembler syntax used by the reference's JSON test
// vectors (src/core_read.cpp ParseScript): decimal numbers, 0x raw hex, 'quoted strings' and
// opcode names with or without the OP_ prefix.
CScript ParseScript(const std::string& s);
std::string ScriptToAsmStr(const CScript& script, bool fAttemptSighashDecode = false);

} // namespace bcp
