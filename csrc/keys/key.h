// Keys, public keys, BIP32 extended keys, addresses (Base58Check and CashAddr).
// Parity: reference src/pubkey.{h,cpp} (CPubKey incl. Verify/RecoverCompact/Derive,
// CExtPubKey), src/key.{h,cpp} (CKey::Sign with RFC6979 + test_case entropy,
// SignCompact, Derive, CExtKey::SetMaster "Bitcoin seed"), src/base58.{h,cpp},
// src/cashaddr.cpp + src/cashaddrenc.cpp, src/dstencode.cpp.
#pragma once
#include "primitives/uint256.h"
#include "crypto/hashes.h"
#include "script/script.h"
#include "util/lockedpool.h"

#include <string>
#include <vector>

namespace bcp {

class CChainParams;

typedef uint256 ChainCode;
class CKeyID : public uint160 {
public:
    CKeyID() {}
    explicit CKeyID(const uint160& in) : uint160(in) {}
};
class CScriptID : public uint160 {
public:
    CScriptID() {}
    explicit CScriptID(const CScript& in);
    explicit CScriptID(const uint160& in) : uint160(in) {}
};

class CPubKey {
public:
    static const unsigned int PUBLIC_KEY_SIZE = 65;
    static const unsigned int COMPRESSED_PUBLIC_KEY_SIZE = 33;
    static const unsigned int SIGNATURE_SIZE = 72;
    static const unsigned int COMPACT_SIGNATURE_SIZE = 65;

    CPubKey() {}
    template <typename It> CPubKey(It b, It e) { Set(b, e); }
    explicit CPubKey(const std::vector<unsigned char>& v) { Set(v.begin(), v.end()); }
    template <typename It> void Set(It b, It e) {
        vch.assign(b, e);
        if (vch.empty() || GetLen(vch[0]) != vch.size()) vch.clear();
    }
    static unsigned int GetLen(unsigned char chHeader) {
        if (chHeader == 2 || chHeader == 3) return COMPRESSED_PUBLIC_KEY_SIZE;
        if (chHeader == 4 || chHeader == 6 || chHeader == 7) return PUBLIC_KEY_SIZE;
        return 0;
    }
    size_t size() const { return vch.size(); }
    const unsigned char* begin() const { return vch.data(); }
    const unsigned char* end() const { return vch.data() + vch.size(); }
    const unsigned char& operator[](unsigned int pos) const { return vch[pos]; }
    const std::vector<unsigned char>& Raw() const { return vch; }
    friend bool operator==(const CPubKey& a, const CPubKey& b) { return a.vch == b.vch; }
    friend bool operator!=(const CPubKey& a, const CPubKey& b) { return a.vch != b.vch; }
    friend bool operator<(const CPubKey& a, const CPubKey& b) { return a.vch < b.vch; }

    CKeyID GetID() const;
    uint256 GetHash() const;
    bool IsValid() const { return !vch.empty(); }
    bool IsFullyValid() const;
    bool IsCompressed() const { return vch.size() == COMPRESSED_PUBLIC_KEY_SIZE; }
    // CPubKey::Verify semantics: lax DER, low-S normalised, then verify.
    bool Verify(const uint256& hash, const std::vector<unsigned char>& vchSig) const;
    static bool CheckLowS(const std::vector<unsigned char>& vchSig);
    bool RecoverCompact(const uint256& hash, const std::vector<unsigned char>& vchSig);
    bool Decompress();
    bool Derive(CPubKey& pubkeyChild, ChainCode& ccChild, unsigned int nChild, const ChainCode& cc) const;

    template <typename S> void Serialize(S& s) const { ::bcp::Serialize(s, vch); }
    template <typename S> void Unserialize(S& s) {
        std::vector<unsigned char> v;
        ::bcp::Unserialize(s, v);
        Set(v.begin(), v.end());
    }

private:
    std::vector<unsigned char> vch;
};

// Private key bytes in locked, cleansed-on-free memory (reference src/key.h:32 CPrivKey).
typedef std::vector<unsigned char, secure_allocator<unsigned char>> CPrivKey;

// The 32 secret bytes live in the process's LockedPool (mlocked pages, cleansed when freed), as
// the reference's CKey::keydata does (src/key.h:47); copies of a key allocate their own.
class CKey {
public:
    CKey() : keydata(32) {}
    bool IsValid() const { return fValid; }
    bool IsCompressed() const { return fCompressed; }
    const unsigned char* begin() const { return keydata.data(); }
    const unsigned char* end() const { return keydata.data() + 32; }
    unsigned int size() const { return fValid ? 32 : 0; }
    friend bool operator==(const CKey& a, const CKey& b) {
        return a.fCompressed == b.fCompressed && a.fValid == b.fValid && memcmp(a.begin(), b.begin(), 32) == 0;
    }
    template <typename It> void Set(It b, It e, bool compressed) {
        if ((size_t)(e - b) != 32) {
            fValid = false;
            return;
        }
        std::copy(b, e, keydata.begin());
        fValid = Check(keydata.data());
        fCompressed = compressed;
    }
    static bool Check(const unsigned char* vch);
    void MakeNewKey(bool fCompressed);
    CPubKey GetPubKey() const;
    // DER signature, low-S. test_case != 0 adds extra entropy (reference CKey::Sign).
    bool Sign(const uint256& hash, std::vector<unsigned char>& vchSig, uint32_t test_case = 0) const;
    bool SignCompact(const uint256& hash, std::vector<unsigned char>& vchSig) const;
    bool Derive(CKey& keyChild, ChainCode& ccChild, unsigned int nChild, const ChainCode& cc) const;
    bool VerifyPubKey(const CPubKey& vchPubKey) const;
    CPrivKey GetPrivKeyBytes() const { return CPrivKey(keydata.begin(), keydata.end()); }

private:
    bool fValid = false;
    bool fCompressed = false;
    CPrivKey keydata;
};

static const unsigned int BIP32_EXTKEY_SIZE = 74;
void BIP32Hash(const ChainCode& chainCode, unsigned int nChild, unsigned char header, const unsigned char data[32],
               unsigned char output[64]);

struct CExtPubKey {
    unsigned char nDepth = 0;
    unsigned char vchFingerprint[4] = {0, 0, 0, 0};
    unsigned int nChild = 0;
    ChainCode chaincode;
    CPubKey pubkey;
    void Encode(unsigned char code[BIP32_EXTKEY_SIZE]) const;
    void Decode(const unsigned char code[BIP32_EXTKEY_SIZE]);
    bool Derive(CExtPubKey& out, unsigned int nChild) const;
};

struct CExtKey {
    unsigned char nDepth = 0;
    unsigned char vchFingerprint[4] = {0, 0, 0, 0};
    unsigned int nChild = 0;
    ChainCode chaincode;
    CKey key;
    void Encode(unsigned char code[BIP32_EXTKEY_SIZE]) const;
    void Decode(const unsigned char code[BIP32_EXTKEY_SIZE]);
    bool Derive(CExtKey& out, unsigned int nChild) const;
    CExtPubKey Neuter() const;
    void SetMaster(const unsigned char* seed, unsigned int nSeedLen);
};

// ---------------------------------------------------------------- random
void GetRandBytes(unsigned char* buf, size_t num);
void GetStrongRandBytes(unsigned char* buf, size_t num);
// Start-up checks (reference init.cpp InitSanityCheck): a fresh key's public key verifies
// against it (ECC_InitSanityCheck, key.cpp:336), and the OS RNG overwrites every byte of a
// 32-byte buffer within 1024 reads (Random_SanityCheck, random.cpp:253).
bool ECC_InitSanityCheck();
bool Random_SanityCheck();
uint64_t GetRand(uint64_t nMax);
int GetRandInt(int nMax);
uint256 GetRandHash();
class FastRandomContext {
public:
    explicit FastRandomContext(bool fDeterministic = false);
    explicit FastRandomContext(const uint256& seed);
    uint64_t rand64();
    uint64_t randbits(int bits); // bits in [0, 64]
    std::vector<unsigned char> randbytes(size_t len);
    uint32_t rand32() { return (uint32_t)rand64(); }
    uint64_t randrange(uint64_t range);
    bool randbool() { return rand64() & 1; }
    uint256 rand256();
private:
    void Fill();
    ChaCha20 rng;
    unsigned char buf[64];
    int avail = 0;
};

// ---------------------------------------------------------------- encodings
std::string EncodeBase58(const unsigned char* pbegin, const unsigned char* pend);
std::string EncodeBase58(const std::vector<unsigned char>& vch);
bool DecodeBase58(const std::string& str, std::vector<unsigned char>& vchRet);
std::string EncodeBase58Check(const std::vector<unsigned char>& vchIn);
bool DecodeBase58Check(const std::string& str, std::vector<unsigned char>& vchRet);

namespace cashaddr {
std::string Encode(const std::string& prefix, const std::vector<uint8_t>& values);
std::pair<std::string, std::vector<uint8_t>> Decode(const std::string& str, const std::string& default_prefix);
} // namespace cashaddr

// Destinations
enum class DestType { NONE, KEYID, SCRIPTID };
struct CTxDestination {
    DestType type = DestType::NONE;
    uint160 hash;
    CTxDestination() {}
    CTxDestination(const CKeyID& id) : type(DestType::KEYID), hash(id) {}
    CTxDestination(const CScriptID& id) : type(DestType::SCRIPTID), hash(id) {}
    bool IsValid() const { return type != DestType::NONE; }
    friend bool operator==(const CTxDestination& a, const CTxDestination& b) { return a.type == b.type && a.hash == b.hash; }
    friend bool operator<(const CTxDestination& a, const CTxDestination& b) {
        return a.type < b.type || (a.type == b.type && a.hash < b.hash);
    }
};

std::string EncodeLegacyAddr(const CTxDestination& dest, const CChainParams& params);
CTxDestination DecodeLegacyAddr(const std::string& str, const CChainParams& params);
std::string EncodeCashAddr(const CTxDestination& dest, const CChainParams& params);
CTxDestination DecodeCashAddr(const std::string& str, const CChainParams& params);
// dstencode: -usecashaddr selects the output format; decoding accepts both.
void SetUseCashAddr(bool on);
bool UseCashAddr();
std::string EncodeDestination(const CTxDestination& dest, const CChainParams& params);
CTxDestination DecodeDestination(const std::string& str, const CChainParams& params);
bool IsValidDestinationString(const std::string& str, const CChainParams& params);

std::string EncodeSecret(const CKey& key, const CChainParams& params);
CKey DecodeSecret(const std::string& str, const CChainParams& params);
std::string EncodeExtKey(const CExtKey& key, const CChainParams& params);
CExtKey DecodeExtKey(const std::string& str, const CChainParams& params);
std::string EncodeExtPubKey(const CExtPubKey& key, const CChainParams& params);
CExtPubKey DecodeExtPubKey(const std::string& str, const CChainParams& params);

// Message signing (reference src/rpc/misc.cpp verifymessage/signmessagewithprivkey).
extern const std::string strMessageMagic;
uint256 MessageHash(const std::string& message);

} // namespace bcp
