// Script container implementation (reference src/script/script.cpp, src/core_read.cpp ParseScript,
// src/core_write.cpp ScriptToAsmStr).
#include "script/script.h"
#include "util/strencodings.h"

#include <cctype>
#include <cstring>
#include <map>

namespace bcp {

const char* GetOpName(opcodetype opcode) {
    switch (opcode) {
    case OP_0: return "0";
    case OP_PUSHDATA1: return "OP_PUSHDATA1";
    case OP_PUSHDATA2: return "OP_PUSHDATA2";
    case OP_PUSHDATA4: return "OP_PUSHDATA4";
    case OP_1NEGATE: return "-1";
    case OP_RESERVED: return "OP_RESERVED";
    case OP_1: return "1";
    case OP_2: return "2";
    case OP_3: return "3";
    case OP_4: return "4";
    case OP_5: return "5";
    case OP_6: return "6";
    case OP_7: return "7";
    case OP_8: return "8";
    case OP_9: return "9";
    case OP_10: return "10";
    case OP_11: return "11";
    case OP_12: return "12";
    case OP_13: return "13";
    case OP_14: return "14";
    case OP_15: return "15";
    case OP_16: return "16";
    case OP_NOP: return "OP_NOP";
    case OP_VER: return "OP_VER";
    case OP_IF: return "OP_IF";
    case OP_NOTIF: return "OP_NOTIF";
    case OP_VERIF: return "OP_VERIF";
    case OP_VERNOTIF: return "OP_VERNOTIF";
    case OP_ELSE: return "OP_ELSE";
    case OP_ENDIF: return "OP_ENDIF";
    case OP_VERIFY: return "OP_VERIFY";
    case OP_RETURN: return "OP_RETURN";
    case OP_TOALTSTACK: return "OP_TOALTSTACK";
    case OP_FROMALTSTACK: return "OP_FROMALTSTACK";
    case OP_2DROP: return "OP_2DROP";
    case OP_2DUP: return "OP_2DUP";
    case OP_3DUP: return "OP_3DUP";
    case OP_2OVER: return "OP_2OVER";
    case OP_2ROT: return "OP_2ROT";
    case OP_2SWAP: return "OP_2SWAP";
    case OP_IFDUP: return "OP_IFDUP";
    case OP_DEPTH: return "OP_DEPTH";
    case OP_DROP: return "OP_DROP";
    case OP_DUP: return "OP_DUP";
    case OP_NIP: return "OP_NIP";
    case OP_OVER: return "OP_OVER";
    case OP_PICK: return "OP_PICK";
    case OP_ROLL: return "OP_ROLL";
    case OP_ROT: return "OP_ROT";
    case OP_SWAP: return "OP_SWAP";
    case OP_TUCK: return "OP_TUCK";
    case OP_CAT: return "OP_CAT";
    case OP_SUBSTR: return "OP_SUBSTR";
    case OP_LEFT: return "OP_LEFT";
    case OP_RIGHT: return "OP_RIGHT";
    case OP_SIZE: return "OP_SIZE";
    case OP_INVERT: return "OP_INVERT";
    case OP_AND: return "OP_AND";
    case OP_OR: return "OP_OR";
    case OP_XOR: return "OP_XOR";
    case OP_EQUAL: return "OP_EQUAL";
    case OP_EQUALVERIFY: return "OP_EQUALVERIFY";
    case OP_RESERVED1: return "OP_RESERVED1";
    case OP_RESERVED2: return "OP_RESERVED2";
    case OP_1ADD: return "OP_1ADD";
    case OP_1SUB: return "OP_1SUB";
    case OP_2MUL: return "OP_2MUL";
    case OP_2DIV: return "OP_2DIV";
    case OP_NEGATE: return "OP_NEGATE";
    case OP_ABS: return "OP_ABS";
    case OP_NOT: return "OP_NOT";
    case OP_0NOTEQUAL: return "OP_0NOTEQUAL";
    case OP_ADD: return "OP_ADD";
    case OP_SUB: return "OP_SUB";
    case OP_MUL: return "OP_MUL";
    case OP_DIV: return "OP_DIV";
    case OP_MOD: return "OP_MOD";
    case OP_LSHIFT: return "OP_LSHIFT";
    case OP_RSHIFT: return "OP_RSHIFT";
    case OP_BOOLAND: return "OP_BOOLAND";
    case OP_BOOLOR: return "OP_BOOLOR";
    case OP_NUMEQUAL: return "OP_NUMEQUAL";
    case OP_NUMEQUALVERIFY: return "OP_NUMEQUALVERIFY";
    case OP_NUMNOTEQUAL: return "OP_NUMNOTEQUAL";
    case OP_LESSTHAN: return "OP_LESSTHAN";
    case OP_GREATERTHAN: return "OP_GREATERTHAN";
    case OP_LESSTHANOREQUAL: return "OP_LESSTHANOREQUAL";
    case OP_GREATERTHANOREQUAL: return "OP_GREATERTHANOREQUAL";
    case OP_MIN: return "OP_MIN";
    case OP_MAX: return "OP_MAX";
    case OP_WITHIN: return "OP_WITHIN";
    case OP_RIPEMD160: return "OP_RIPEMD160";
    case OP_SHA1: return "OP_SHA1";
    case OP_SHA256: return "OP_SHA256";
    case OP_HASH160: return "OP_HASH160";
    case OP_HASH256: return "OP_HASH256";
    case OP_CODESEPARATOR: return "OP_CODESEPARATOR";
    case OP_CHECKSIG: return "OP_CHECKSIG";
    case OP_CHECKSIGVERIFY: return "OP_CHECKSIGVERIFY";
    case OP_CHECKMULTISIG: return "OP_CHECKMULTISIG";
    case OP_CHECKMULTISIGVERIFY: return "OP_CHECKMULTISIGVERIFY";
    case OP_NOP1: return "OP_NOP1";
    case OP_CHECKLOCKTIMEVERIFY: return "OP_CHECKLOCKTIMEVERIFY";
    case OP_CHECKSEQUENCEVERIFY: return "OP_CHECKSEQUENCEVERIFY";
    case OP_NOP4: return "OP_NOP4";
    case OP_NOP5: return "OP_NOP5";
    case OP_NOP6: return "OP_NOP6";
    case OP_NOP7: return "OP_NOP7";
    case OP_NOP8: return "OP_NOP8";
    case OP_NOP9: return "OP_NOP9";
    case OP_NOP10: return "OP_NOP10";
    case OP_INVALIDOPCODE: return "OP_INVALIDOPCODE";
    default: return "OP_UNKNOWN";
    }
}

CScriptNum::CScriptNum(const std::vector<unsigned char>& vch, bool fRequireMinimal, const size_t nMaxNumSize) {
    if (vch.size() > nMaxNumSize) throw scriptnum_error("script number overflow");
    if (fRequireMinimal && !IsMinimallyEncoded(vch, nMaxNumSize)) throw scriptnum_error("non-minimally encoded script number");
    if (vch.empty()) {
        m_value = 0;
        return;
    }
    int64_t result = 0;
    for (size_t i = 0; i != vch.size(); ++i) result |= (int64_t)vch[i] << (8 * i);
    if (vch.back() & 0x80) {
        m_value = -((int64_t)(result & ~(0x80ULL << (8 * (vch.size() - 1)))));
        return;
    }
    m_value = result;
}

bool CScriptNum::IsMinimallyEncoded(const std::vector<unsigned char>& vch, size_t maxSize) {
    if (vch.size() > maxSize) return false;
    if (vch.size() > 0) {
        // The most significant byte may not be 0x00 or 0x80 unless the next byte's high bit is set.
        if ((vch.back() & 0x7f) == 0) {
            if (vch.size() <= 1 || (vch[vch.size() - 2] & 0x80) == 0) return false;
        }
    }
    return true;
}

std::vector<unsigned char> CScriptNum::serialize(const int64_t& value) {
    if (value == 0) return {};
    std::vector<unsigned char> result;
    const bool neg = value < 0;
    uint64_t absvalue = neg ? (uint64_t)(-(value + 1)) + 1 : (uint64_t)value;
    while (absvalue) {
        result.push_back(absvalue & 0xff);
        absvalue >>= 8;
    }
    if (result.back() & 0x80) result.push_back(neg ? 0x80 : 0);
    else if (neg) result.back() |= 0x80;
    return result;
}

CScript& CScript::operator<<(const std::vector<unsigned char>& b) {
    if (b.size() < OP_PUSHDATA1) {
        insert(end(), (unsigned char)b.size());
    } else if (b.size() <= 0xff) {
        insert(end(), OP_PUSHDATA1);
        insert(end(), (unsigned char)b.size());
    } else if (b.size() <= 0xffff) {
        insert(end(), OP_PUSHDATA2);
        unsigned char d[2] = {(unsigned char)b.size(), (unsigned char)(b.size() >> 8)};
        insert(end(), d, d + 2);
    } else {
        insert(end(), OP_PUSHDATA4);
        uint32_t n = (uint32_t)b.size();
        unsigned char d[4];
        memcpy(d, &n, 4);
        insert(end(), d, d + 4);
    }
    insert(end(), b.begin(), b.end());
    return *this;
}

static bool GetScriptOp(CScript::const_iterator& pc, CScript::const_iterator end, opcodetype& opcodeRet,
                        std::vector<unsigned char>* pvchRet) {
    opcodeRet = OP_INVALIDOPCODE;
    if (pvchRet) pvchRet->clear();
    if (pc >= end) return false;
    if (end - pc < 1) return false;
    unsigned int opcode = *pc++;
    if (opcode <= OP_PUSHDATA4) {
        unsigned int nSize = 0;
        if (opcode < OP_PUSHDATA1) {
            nSize = opcode;
        } else if (opcode == OP_PUSHDATA1) {
            if (end - pc < 1) return false;
            nSize = *pc++;
        } else if (opcode == OP_PUSHDATA2) {
            if (end - pc < 2) return false;
            nSize = pc[0] | (pc[1] << 8);
            pc += 2;
        } else if (opcode == OP_PUSHDATA4) {
            if (end - pc < 4) return false;
            nSize = pc[0] | (pc[1] << 8) | (pc[2] << 16) | ((unsigned int)pc[3] << 24);
            pc += 4;
        }
        if (end - pc < 0 || (unsigned int)(end - pc) < nSize) return false;
        if (pvchRet) pvchRet->assign(pc, pc + nSize);
        pc += nSize;
    }
    opcodeRet = (opcodetype)opcode;
    return true;
}

bool CScript::GetOp(const_iterator& pc, opcodetype& opcodeRet, std::vector<unsigned char>& vchRet) const {
    return GetScriptOp(pc, end(), opcodeRet, &vchRet);
}
bool CScript::GetOp(const_iterator& pc, opcodetype& opcodeRet) const {
    return GetScriptOp(pc, end(), opcodeRet, nullptr);
}

unsigned int CScript::GetSigOpCount(bool fAccurate) const {
    unsigned int n = 0;
    const_iterator pc = begin();
    opcodetype lastOpcode = OP_INVALIDOPCODE;
    while (pc < end()) {
        opcodetype opcode;
        if (!GetOp(pc, opcode)) break;
        if (opcode == OP_CHECKSIG || opcode == OP_CHECKSIGVERIFY) {
            n++;
        } else if (opcode == OP_CHECKMULTISIG || opcode == OP_CHECKMULTISIGVERIFY) {
            if (fAccurate && lastOpcode >= OP_1 && lastOpcode <= OP_16) n += DecodeOP_N(lastOpcode);
            else n += MAX_PUBKEYS_PER_MULTISIG;
        }
        lastOpcode = opcode;
    }
    return n;
}

unsigned int CScript::GetSigOpCount(const CScript& scriptSig) const {
    if (!IsPayToScriptHash()) return GetSigOpCount(true);
    const_iterator pc = scriptSig.begin();
    std::vector<unsigned char> data;
    while (pc < scriptSig.end()) {
        opcodetype opcode;
        if (!scriptSig.GetOp(pc, opcode, data)) return 0;
        if (opcode > OP_16) return 0;
    }
    CScript subscript(data.begin(), data.end());
    return subscript.GetSigOpCount(true);
}

bool CScript::IsPayToScriptHash() const {
    return size() == 23 && (*this)[0] == OP_HASH160 && (*this)[1] == 0x14 && (*this)[22] == OP_EQUAL;
}

bool CScript::IsPushOnly(const_iterator pc) const {
    while (pc < end()) {
        opcodetype opcode;
        if (!GetOp(pc, opcode)) return false;
        if (opcode > OP_16) return false;
    }
    return true;
}

bool CScript::IsCommitment(const std::vector<unsigned char>& data) const {
    if (data.size() > 64 || size() != data.size() + 2) return false;
    if ((*this)[0] != OP_RETURN || (*this)[1] != data.size()) return false;
    return memcmp(this->data() + 2, data.data(), data.size()) == 0;
}

int CScript::FindAndDelete(const CScript& b) {
    int nFound = 0;
    if (b.empty()) return nFound;
    CScript result;
    const_iterator pc = begin(), pc2 = begin();
    opcodetype opcode;
    do {
        result.insert(result.end(), pc2, pc);
        while ((size_t)(end() - pc) >= b.size() && std::equal(b.begin(), b.end(), pc)) {
            pc = pc + b.size();
            ++nFound;
        }
        pc2 = pc;
    } while (GetOp(pc, opcode));
    if (nFound > 0) {
        result.insert(result.end(), pc2, cend());
        *this = result;
    }
    return nFound;
}

std::string CScript::ToString() const {
    std::string str;
    opcodetype opcode;
    std::vector<unsigned char> vch;
    const_iterator pc = begin();
    while (pc < end()) {
        if (!str.empty()) str += " ";
        if (!GetOp(pc, opcode, vch)) {
            str += "[error]";
            return str;
        }
        if (0 <= opcode && opcode <= OP_PUSHDATA4) {
            if (vch.size() <= 4) str += std::to_string(CScriptNum(vch, false).getint64());
            else str += HexStr(vch);
        } else {
            str += GetOpName(opcode);
        }
    }
    return str;
}

CScript ParseScript(const std::string& s) {
    static std::map<std::string, opcodetype> mapOpNames;
    if (mapOpNames.empty()) {
        for (int op = 0; op <= OP_NOP10; op++) {
            if (op < OP_NOP && op != OP_RESERVED) continue;
            const char* name = GetOpName((opcodetype)op);
            if (strcmp(name, "OP_UNKNOWN") == 0) continue;
            std::string strName(name);
            mapOpNames[strName] = (opcodetype)op;
            if (strName.rfind("OP_", 0) == 0) mapOpNames[strName.substr(3)] = (opcodetype)op;
        }
    }
    CScript result;
    std::vector<std::string> words;
    std::string cur;
    for (char c : s) {
        if (c == ' ' || c == '\t' || c == '\n') {
            if (!cur.empty()) words.push_back(cur);
            cur.clear();
        } else {
            cur.push_back(c);
        }
    }
    if (!cur.empty()) words.push_back(cur);
    auto all_digits = [](const std::string& w, size_t from) {
        if (w.size() <= from) return false;
        for (size_t i = from; i < w.size(); ++i)
            if (!isdigit((unsigned char)w[i])) return false;
        return true;
    };
    for (const std::string& w : words) {
        if (all_digits(w, 0) || (w[0] == '-' && all_digits(w, 1))) {
            result << atoi64(w);
        } else if (w.rfind("0x", 0) == 0 && w.size() > 2 && IsHex(w.substr(2))) {
            std::vector<unsigned char> raw = ParseHex(w.substr(2));
            result.insert(result.end(), raw.begin(), raw.end());
        } else if (w.size() >= 2 && w.front() == '\'' && w.back() == '\'') {
            std::vector<unsigned char> value(w.begin() + 1, w.end() - 1);
            result << value;
        } else if (mapOpNames.count(w)) {
            result << mapOpNames[w];
        } else {
            throw std::runtime_error("script parse error");
        }
    }
    return result;
}

std::string ScriptToAsmStr(const CScript& script, bool fAttemptSighashDecode) {
    std::string str;
    opcodetype opcode;
    std::vector<unsigned char> vch;
    CScript::const_iterator pc = script.begin();
    while (pc < script.end()) {
        if (!str.empty()) str += " ";
        if (!script.GetOp(pc, opcode, vch)) {
            str += "[error]";
            return str;
        }
        if (0 <= opcode && opcode <= OP_PUSHDATA4) {
            if (vch.size() <= 4) {
                str += std::to_string(CScriptNum(vch, false).getint64());
            } else {
                if (fAttemptSighashDecode && !script.IsUnspendable() && vch.size() >= 9 && vch[0] == 0x30) {
                    // signature: DER || hashtype
                    const unsigned char ht = vch.back();
                    static const std::map<unsigned char, std::string> names = {
                        {0x01, "ALL"}, {0x02, "NONE"}, {0x03, "SINGLE"}, {0x81, "ALL|ANYONECANPAY"},
                        {0x82, "NONE|ANYONECANPAY"}, {0x83, "SINGLE|ANYONECANPAY"}, {0x41, "ALL|FORKID"},
                        {0x42, "NONE|FORKID"}, {0x43, "SINGLE|FORKID"}, {0xc1, "ALL|FORKID|ANYONECANPAY"},
                        {0xc2, "NONE|FORKID|ANYONECANPAY"}, {0xc3, "SINGLE|FORKID|ANYONECANPAY"}};
                    auto it = names.find(ht);
                    if (it != names.end()) {
                        str += HexStr(vch.data(), vch.data() + vch.size() - 1) + "[" + it->second + "]";
                        continue;
                    }
                }
                str += HexStr(vch);
            }
        } else {
            str += GetOpName(opcode);
        }
    }
    return str;
}

} // namespace bcp
