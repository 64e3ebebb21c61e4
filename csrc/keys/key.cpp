// Keys, BIP32, randomness, Base58Check / CashAddr address encodings.
// Parity notes (reference file:line):
//   CKey::Sign test_case entropy   src/key.cpp:196-210
//   CKey::SignCompact header byte  src/key.cpp:228-245  (27 + recid + 4*compressed)
//   CKey::Derive / BIP32Hash       src/key.cpp:277-300, src/hash.cpp:73-84
//   CExtKey::SetMaster "Bitcoin seed" src/key.cpp:310-320
//   CPubKey::RecoverCompact        src/pubkey.cpp:195-215
//   Base58                         src/base58.cpp:20-120
//   CashAddr polymod / charset     src/cashaddr.cpp:20-200, src/cashaddrenc.cpp:20-180
//   dstencode                      src/dstencode.cpp:10-40
#include "keys/key.h"
#include "consensus/params.h"
#include "crypto/common.h"
#include "secp256k1/secp256k1.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <fcntl.h>
#include <mutex>
#include <stdexcept>
#include <unistd.h>

namespace bcp {

CScriptID::CScriptID(const CScript& in) : uint160(Hash160(in)) {}

// ------------------------------------------------------------------ CPubKey
CKeyID CPubKey::GetID() const { return CKeyID(Hash160(vch)); }
uint256 CPubKey::GetHash() const { return Hash256(vch); }

bool CPubKey::IsFullyValid() const {
    if (!IsValid()) return false;
    secp::Ge p;
    return secp::pubkey_parse(p, vch.data(), vch.size());
}

bool CPubKey::Verify(const uint256& hash, const std::vector<unsigned char>& vchSig) const {
    if (!IsValid()) return false;
    return secp::VerifySignature(vch.data(), vch.size(), vchSig.data(), vchSig.size(), hash.begin());
}

bool CPubKey::CheckLowS(const std::vector<unsigned char>& vchSig) {
    secp::Signature sig;
    if (!secp::sig_parse_der_lax(sig, vchSig.data(), vchSig.size())) return false;
    return !secp::sig_normalize(sig);
}

bool CPubKey::RecoverCompact(const uint256& hash, const std::vector<unsigned char>& vchSig) {
    if (vchSig.size() != COMPACT_SIGNATURE_SIZE) return false;
    const int hdr = vchSig[0] - 27;
    if (hdr < 0 || hdr > 7) return false;
    const int recid = hdr & 3;
    const bool comp = (hdr & 4) != 0;
    secp::Signature sig;
    if (!secp::sig_parse_compact(sig, &vchSig[1])) return false;
    secp::Ge p;
    if (!secp::ecdsa_recover(p, sig, recid, hash.begin())) return false;
    std::vector<unsigned char> ser = secp::pubkey_serialize(p, comp);
    Set(ser.begin(), ser.end());
    return true;
}

bool CPubKey::Decompress() {
    if (!IsValid()) return false;
    secp::Ge p;
    if (!secp::pubkey_parse(p, vch.data(), vch.size())) return false;
    std::vector<unsigned char> ser = secp::pubkey_serialize(p, false);
    Set(ser.begin(), ser.end());
    return true;
}

bool CPubKey::Derive(CPubKey& pubkeyChild, ChainCode& ccChild, unsigned int nChild, const ChainCode& cc) const {
    if (!IsValid() || (nChild >> 31) != 0 || size() != COMPRESSED_PUBLIC_KEY_SIZE) return false;
    unsigned char out[64];
    BIP32Hash(cc, nChild, vch[0], vch.data() + 1, out);
    memcpy(ccChild.begin(), out + 32, 32);
    secp::Ge p;
    if (!secp::pubkey_parse(p, vch.data(), vch.size())) return false;
    if (!secp::pubkey_tweak_add(p, out)) return false;
    std::vector<unsigned char> ser = secp::pubkey_serialize(p, true);
    pubkeyChild.Set(ser.begin(), ser.end());
    return true;
}

// ------------------------------------------------------------------ CKey
bool CKey::Check(const unsigned char* vch) { return secp::seckey_verify(vch); }

void CKey::MakeNewKey(bool compressed) {
    do {
        GetStrongRandBytes(keydata.data(), 32);
    } while (!Check(keydata.data()));
    fValid = true;
    fCompressed = compressed;
}

CPubKey CKey::GetPubKey() const {
    if (!fValid) throw std::logic_error("CKey::GetPubKey on invalid key");
    secp::Ge p;
    if (!secp::pubkey_create(p, keydata.data())) throw std::logic_error("pubkey_create failed");
    std::vector<unsigned char> ser = secp::pubkey_serialize(p, fCompressed);
    return CPubKey(ser);
}

bool CKey::Sign(const uint256& hash, std::vector<unsigned char>& vchSig, uint32_t test_case) const {
    if (!fValid) return false;
    unsigned char extra[32] = {0};
    WriteLE32(extra, test_case);
    secp::Signature sig;
    int recid = 0;
    if (!secp::ecdsa_sign(sig, &recid, hash.begin(), keydata.data(), test_case ? extra : nullptr)) return false;
    vchSig = secp::sig_serialize_der(sig);
    return true;
}

bool CKey::SignCompact(const uint256& hash, std::vector<unsigned char>& vchSig) const {
    if (!fValid) return false;
    secp::Signature sig;
    int recid = 0;
    if (!secp::ecdsa_sign(sig, &recid, hash.begin(), keydata.data(), nullptr)) return false;
    vchSig.assign(CPubKey::COMPACT_SIGNATURE_SIZE, 0);
    secp::sig_serialize_compact(&vchSig[1], sig);
    vchSig[0] = (unsigned char)(27 + recid + (fCompressed ? 4 : 0));
    return true;
}

bool CKey::VerifyPubKey(const CPubKey& pubkey) const {
    if (pubkey.IsCompressed() != fCompressed) return false;
    static const std::string str = "Bitcoin key verification\n";
    unsigned char rnd[8];
    GetRandBytes(rnd, sizeof(rnd));
    CSHA256 h;
    h.Write((const unsigned char*)str.data(), str.size()).Write(rnd, sizeof(rnd));
    uint256 hash;
    h.Finalize(hash.begin());
    CSHA256().Write(hash.begin(), 32).Finalize(hash.begin());
    std::vector<unsigned char> sig;
    Sign(hash, sig);
    return pubkey.Verify(hash, sig);
}

bool CKey::Derive(CKey& keyChild, ChainCode& ccChild, unsigned int nChild, const ChainCode& cc) const {
    if (!fValid) return false;
    unsigned char out[64];
    if ((nChild >> 31) == 0) {
        secp::Ge p;
        if (!secp::pubkey_create(p, keydata.data())) return false;
        std::vector<unsigned char> pub = secp::pubkey_serialize(p, true);
        BIP32Hash(cc, nChild, pub[0], pub.data() + 1, out);
    } else {
        BIP32Hash(cc, nChild, 0, keydata.data(), out);
    }
    memcpy(ccChild.begin(), out + 32, 32);
    memcpy(keyChild.keydata.data(), keydata.data(), 32);
    const bool ok = secp::seckey_tweak_add(keyChild.keydata.data(), out);
    memory_cleanse(out, sizeof(out));
    keyChild.fCompressed = true;
    keyChild.fValid = ok;
    return ok;
}

void BIP32Hash(const ChainCode& chainCode, unsigned int nChild, unsigned char header, const unsigned char data[32],
               unsigned char output[64]) {
    unsigned char num[4];
    WriteBE32(num, nChild);
    CHMAC_SHA512(chainCode.begin(), 32).Write(&header, 1).Write(data, 32).Write(num, 4).Finalize(output);
}

// ------------------------------------------------------------------ BIP32
static void EncodeExtHeader(unsigned char code[BIP32_EXTKEY_SIZE], unsigned char depth, const unsigned char fp[4],
                            unsigned int child, const ChainCode& cc) {
    code[0] = depth;
    memcpy(code + 1, fp, 4);
    WriteBE32(code + 5, child);
    memcpy(code + 9, cc.begin(), 32);
}

void CExtPubKey::Encode(unsigned char code[BIP32_EXTKEY_SIZE]) const {
    EncodeExtHeader(code, nDepth, vchFingerprint, nChild, chaincode);
    if (pubkey.size() != CPubKey::COMPRESSED_PUBLIC_KEY_SIZE) throw std::logic_error("ext pubkey must be compressed");
    memcpy(code + 41, pubkey.begin(), 33);
}
void CExtPubKey::Decode(const unsigned char code[BIP32_EXTKEY_SIZE]) {
    nDepth = code[0];
    memcpy(vchFingerprint, code + 1, 4);
    nChild = ReadBE32(code + 5);
    memcpy(chaincode.begin(), code + 9, 32);
    pubkey.Set(code + 41, code + BIP32_EXTKEY_SIZE);
}
bool CExtPubKey::Derive(CExtPubKey& out, unsigned int child) const {
    out.nDepth = nDepth + 1;
    CKeyID id = pubkey.GetID();
    memcpy(out.vchFingerprint, id.begin(), 4);
    out.nChild = child;
    return pubkey.Derive(out.pubkey, out.chaincode, child, chaincode);
}

void CExtKey::Encode(unsigned char code[BIP32_EXTKEY_SIZE]) const {
    EncodeExtHeader(code, nDepth, vchFingerprint, nChild, chaincode);
    code[41] = 0;
    if (key.size() != 32) throw std::logic_error("ext key invalid");
    memcpy(code + 42, key.begin(), 32);
}
void CExtKey::Decode(const unsigned char code[BIP32_EXTKEY_SIZE]) {
    nDepth = code[0];
    memcpy(vchFingerprint, code + 1, 4);
    nChild = ReadBE32(code + 5);
    memcpy(chaincode.begin(), code + 9, 32);
    key.Set(code + 42, code + BIP32_EXTKEY_SIZE, true);
}
bool CExtKey::Derive(CExtKey& out, unsigned int child) const {
    out.nDepth = nDepth + 1;
    CKeyID id = key.GetPubKey().GetID();
    memcpy(out.vchFingerprint, id.begin(), 4);
    out.nChild = child;
    return key.Derive(out.key, out.chaincode, child, chaincode);
}
CExtPubKey CExtKey::Neuter() const {
    CExtPubKey r;
    r.nDepth = nDepth;
    memcpy(r.vchFingerprint, vchFingerprint, 4);
    r.nChild = nChild;
    r.pubkey = key.GetPubKey();
    r.chaincode = chaincode;
    return r;
}
void CExtKey::SetMaster(const unsigned char* seed, unsigned int nSeedLen) {
    static const unsigned char hashkey[] = {'B', 'i', 't', 'c', 'o', 'i', 'n', ' ', 's', 'e', 'e', 'd'};
    unsigned char I[64];
    CHMAC_SHA512(hashkey, sizeof(hashkey)).Write(seed, nSeedLen).Finalize(I);
    key.Set(I, I + 32, true);
    memcpy(chaincode.begin(), I + 32, 32);
    nDepth = 0;
    nChild = 0;
    memset(vchFingerprint, 0, 4);
    memory_cleanse(I, sizeof(I));
}

// ------------------------------------------------------------------ randomness
// OS entropy is mixed with a process-wide ChaCha20 stream keyed from /dev/urandom
// and the high-resolution clock; GetStrongRandBytes re-reads the OS source.
static void GetOSRand(unsigned char* buf, size_t num) {
    int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open /dev/urandom");
    size_t have = 0;
    while (have < num) {
        ssize_t n = read(fd, buf + have, num - have);
        if (n <= 0) {
            close(fd);
            throw std::runtime_error("read /dev/urandom failed");
        }
        have += (size_t)n;
    }
    close(fd);
}

void GetRandBytes(unsigned char* buf, size_t num) { GetOSRand(buf, num); }

bool Random_SanityCheck() {
    // not a quality test: every byte must change at least once within the try budget
    unsigned char data[32];
    bool overwritten[32] = {};
    int num = 0;
    for (int tries = 0; tries < 1024 && num < 32; tries++) {
        memset(data, 0, sizeof(data));
        GetOSRand(data, sizeof(data));
        num = 0;
        for (int x = 0; x < 32; x++) {
            overwritten[x] |= data[x] != 0;
            num += overwritten[x];
        }
    }
    return num == 32;
}

bool ECC_InitSanityCheck() {
    CKey key;
    key.MakeNewKey(true);
    return key.VerifyPubKey(key.GetPubKey());
}

void GetStrongRandBytes(unsigned char* buf, size_t num) {
    // Hash OS randomness together with a timestamp so a weak OS source alone
    // does not determine the output.
    size_t off = 0;
    while (off < num) {
        unsigned char seed[64];
        GetOSRand(seed, 32);
        const uint64_t t = (uint64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count();
        WriteLE64(seed + 32, t);
        memset(seed + 40, 0, 24);
        unsigned char out[64];
        CSHA512().Write(seed, sizeof(seed)).Finalize(out);
        const size_t n = std::min<size_t>(32, num - off);
        memcpy(buf + off, out, n);
        off += n;
        memory_cleanse(seed, sizeof(seed));
        memory_cleanse(out, sizeof(out));
    }
}

uint64_t GetRand(uint64_t nMax) {
    if (nMax == 0) return 0;
    // Rejection sampling to avoid modulo bias.
    const uint64_t nRange = (std::numeric_limits<uint64_t>::max() / nMax) * nMax;
    uint64_t v = 0;
    do {
        GetRandBytes((unsigned char*)&v, sizeof(v));
    } while (v >= nRange);
    return v % nMax;
}
int GetRandInt(int nMax) { return (int)GetRand((uint64_t)nMax); }
uint256 GetRandHash() {
    uint256 h;
    GetRandBytes(h.begin(), 32);
    return h;
}

FastRandomContext::FastRandomContext(bool fDeterministic) {
    unsigned char key[32] = {0};
    if (!fDeterministic) GetRandBytes(key, 32);
    rng.SetKey(key, 32);
}
FastRandomContext::FastRandomContext(const uint256& seed) { rng.SetKey(seed.begin(), 32); }
void FastRandomContext::Fill() {
    rng.Output(buf, sizeof(buf));
    avail = sizeof(buf);
}
uint64_t FastRandomContext::rand64() {
    if (avail < 8) Fill();
    const uint64_t v = ReadLE64(buf + sizeof(buf) - avail);
    avail -= 8;
    return v;
}
uint64_t FastRandomContext::randbits(int bits) {
    if (bits == 0) return 0;
    return rand64() >> (64 - bits);
}
uint64_t FastRandomContext::randrange(uint64_t range) {
    if (range <= 1) return 0;
    --range;
    int bits = 64 - __builtin_clzll(range);
    while (true) {
        const uint64_t r = rand64() >> (64 - bits);
        if (r <= range) return r;
    }
}
uint256 FastRandomContext::rand256() {
    uint256 r;
    for (int i = 0; i < 4; ++i) WriteLE64(r.begin() + 8 * i, rand64());
    return r;
}
std::vector<unsigned char> FastRandomContext::randbytes(size_t len) {
    std::vector<unsigned char> v(len);
    for (size_t i = 0; i < len; i += 8) {
        const uint64_t x = rand64();
        for (size_t j = 0; j < 8 && i + j < len; ++j) v[i + j] = (unsigned char)(x >> (8 * j));
    }
    return v;
}

// ------------------------------------------------------------------ Base58
static const char* const B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

static int8_t B58Rev(char c) {
    static int8_t table[256];
    static std::once_flag once;
    std::call_once(once, [] {
        memset(table, -1, sizeof(table));
        for (int i = 0; i < 58; ++i) table[(unsigned char)B58[i]] = (int8_t)i;
    });
    return table[(unsigned char)c];
}

std::string EncodeBase58(const unsigned char* pbegin, const unsigned char* pend) {
    size_t zeroes = 0;
    while (pbegin != pend && *pbegin == 0) {
        ++pbegin;
        ++zeroes;
    }
    // log(256)/log(58) ~= 1.37; digits are kept little-endian in base 58.
    std::vector<unsigned char> b58((size_t)(pend - pbegin) * 138 / 100 + 1);
    size_t length = 0;
    for (; pbegin != pend; ++pbegin) {
        int carry = *pbegin;
        size_t i = 0;
        for (; (carry != 0 || i < length) && i < b58.size(); ++i) {
            carry += 256 * b58[i];
            b58[i] = (unsigned char)(carry % 58);
            carry /= 58;
        }
        length = i;
    }
    std::string s(zeroes, '1');
    for (size_t i = length; i-- > 0;) s += B58[b58[i]];
    return s;
}
std::string EncodeBase58(const std::vector<unsigned char>& vch) { return EncodeBase58(vch.data(), vch.data() + vch.size()); }

bool DecodeBase58(const std::string& str, std::vector<unsigned char>& vchRet) {
    vchRet.clear();
    size_t p = 0;
    while (p < str.size() && isspace((unsigned char)str[p])) ++p;
    size_t zeroes = 0;
    while (p < str.size() && str[p] == '1') {
        ++zeroes;
        ++p;
    }
    std::vector<unsigned char> b256((str.size() - p) * 733 / 1000 + 1); // log(58)/log(256)
    size_t length = 0;
    while (p < str.size() && !isspace((unsigned char)str[p])) {
        int carry = B58Rev(str[p]);
        if (carry < 0) return false;
        size_t i = 0;
        for (; (carry != 0 || i < length) && i < b256.size(); ++i) {
            carry += 58 * b256[i];
            b256[i] = (unsigned char)(carry & 0xff);
            carry >>= 8;
        }
        if (carry != 0) return false;
        length = i;
        ++p;
    }
    while (p < str.size() && isspace((unsigned char)str[p])) ++p;
    if (p != str.size()) return false;
    vchRet.assign(zeroes, 0);
    for (size_t i = length; i-- > 0;) vchRet.push_back(b256[i]);
    return true;
}

std::string EncodeBase58Check(const std::vector<unsigned char>& vchIn) {
    std::vector<unsigned char> v(vchIn);
    uint256 h = Hash256(v);
    v.insert(v.end(), h.begin(), h.begin() + 4);
    return EncodeBase58(v);
}

bool DecodeBase58Check(const std::string& str, std::vector<unsigned char>& vchRet) {
    if (!DecodeBase58(str, vchRet) || vchRet.size() < 4) {
        vchRet.clear();
        return false;
    }
    uint256 h = Hash256(vchRet.data(), vchRet.size() - 4);
    if (memcmp(h.begin(), &vchRet[vchRet.size() - 4], 4) != 0) {
        vchRet.clear();
        return false;
    }
    vchRet.resize(vchRet.size() - 4);
    return true;
}

// ------------------------------------------------------------------ CashAddr
namespace cashaddr {
static const char* const CHARSET = "qpzry9x8gf2tvdw0s3jn54khce6mua7l";

static int8_t CharsetRev(unsigned char c) {
    static int8_t table[128];
    static std::once_flag once;
    std::call_once(once, [] {
        memset(table, -1, sizeof(table));
        for (int i = 0; i < 32; ++i) {
            table[(unsigned char)CHARSET[i]] = (int8_t)i;
            table[toupper((unsigned char)CHARSET[i])] = (int8_t)i;
        }
    });
    return c < 128 ? table[c] : -1;
}

// BCH-code checksum over GF(2^5): 40-bit remainder of the polynomial whose
// coefficients are the 5-bit values, modulo the generator
// G(x) = x^8 + {19}x^7 + {3}x^6 + {25}x^5 + {11}x^4 + {25}x^3 + {3}x^2 + {19}x + {1}.
static uint64_t PolyMod(const std::vector<uint8_t>& v) {
    static const uint64_t GEN[5] = {0x98f2bc8e61ULL, 0x79b76d99e2ULL, 0xf33e5fb3c4ULL, 0xae2eabe2a8ULL,
                                    0x1e4f43e470ULL};
    uint64_t c = 1;
    for (uint8_t d : v) {
        const uint8_t c0 = (uint8_t)(c >> 35);
        c = ((c & 0x07ffffffffULL) << 5) ^ d;
        for (int b = 0; b < 5; ++b)
            if (c0 & (1 << b)) c ^= GEN[b];
    }
    return c ^ 1;
}

static std::vector<uint8_t> PrefixValues(const std::string& prefix) {
    std::vector<uint8_t> r;
    r.reserve(prefix.size() + 1);
    for (char ch : prefix) r.push_back((uint8_t)ch & 0x1f);
    r.push_back(0);
    return r;
}

std::string Encode(const std::string& prefix, const std::vector<uint8_t>& values) {
    std::vector<uint8_t> v = PrefixValues(prefix);
    v.insert(v.end(), values.begin(), values.end());
    v.insert(v.end(), 8, 0);
    const uint64_t mod = PolyMod(v);
    std::string s = prefix + ':';
    for (uint8_t x : values) s += CHARSET[x];
    for (int i = 0; i < 8; ++i) s += CHARSET[(mod >> (5 * (7 - i))) & 31];
    return s;
}

std::pair<std::string, std::vector<uint8_t>> Decode(const std::string& str, const std::string& default_prefix) {
    bool lower = false, upper = false, digit = false;
    size_t colon = std::string::npos;
    for (size_t i = 0; i < str.size(); ++i) {
        const unsigned char c = (unsigned char)str[i];
        if (c >= 'a' && c <= 'z') lower = true;
        else if (c >= 'A' && c <= 'Z') upper = true;
        else if (c >= '0' && c <= '9') digit = true;
        else if (c == ':') {
            // A prefix must be letters only, non-empty and appear once.
            if (digit || i == 0 || colon != std::string::npos) return {};
            colon = i;
        } else
            return {};
    }
    if (upper && lower) return {};
    std::string prefix;
    size_t start = 0;
    if (colon == std::string::npos) {
        prefix = default_prefix;
    } else {
        for (size_t i = 0; i < colon; ++i) prefix += (char)tolower((unsigned char)str[i]);
        start = colon + 1;
    }
    std::vector<uint8_t> values;
    values.reserve(str.size() - start);
    for (size_t i = start; i < str.size(); ++i) {
        const int8_t r = CharsetRev((unsigned char)str[i]);
        if (r < 0) return {};
        values.push_back((uint8_t)r);
    }
    if (values.size() < 8) return {};
    std::vector<uint8_t> v = PrefixValues(prefix);
    v.insert(v.end(), values.begin(), values.end());
    if (PolyMod(v) != 0) return {};
    values.resize(values.size() - 8);
    return {prefix, values};
}
} // namespace cashaddr

// Regroup a bit stream from FROM-bit to TO-bit words (big-endian bit order).
template <int FROM, int TO, bool PAD>
static bool RegroupBits(std::vector<uint8_t>& out, const uint8_t* in, size_t n) {
    uint32_t acc = 0;
    int bits = 0;
    const uint32_t maxv = (1u << TO) - 1;
    for (size_t i = 0; i < n; ++i) {
        acc = (acc << FROM) | in[i];
        bits += FROM;
        while (bits >= TO) {
            bits -= TO;
            out.push_back((uint8_t)((acc >> bits) & maxv));
        }
    }
    if (PAD) {
        if (bits) out.push_back((uint8_t)((acc << (TO - bits)) & maxv));
        return true;
    }
    return bits < FROM && ((acc << (TO - bits)) & maxv) == 0;
}

// ------------------------------------------------------------------ destinations
std::string EncodeLegacyAddr(const CTxDestination& dest, const CChainParams& params) {
    if (!dest.IsValid()) return "";
    std::vector<unsigned char> d =
        params.Base58Prefix(dest.type == DestType::KEYID ? CChainParams::PUBKEY_ADDRESS : CChainParams::SCRIPT_ADDRESS);
    d.insert(d.end(), dest.hash.begin(), dest.hash.end());
    return EncodeBase58Check(d);
}

CTxDestination DecodeLegacyAddr(const std::string& str, const CChainParams& params) {
    std::vector<unsigned char> d;
    if (!DecodeBase58Check(str, d)) return CTxDestination();
    const auto& pk = params.Base58Prefix(CChainParams::PUBKEY_ADDRESS);
    const auto& sc = params.Base58Prefix(CChainParams::SCRIPT_ADDRESS);
    uint160 h;
    if (d.size() == 20 + pk.size() && std::equal(pk.begin(), pk.end(), d.begin())) {
        memcpy(h.begin(), d.data() + pk.size(), 20);
        return CKeyID(h);
    }
    if (d.size() == 20 + sc.size() && std::equal(sc.begin(), sc.end(), d.begin())) {
        memcpy(h.begin(), d.data() + sc.size(), 20);
        return CScriptID(h);
    }
    return CTxDestination();
}

std::string EncodeCashAddr(const CTxDestination& dest, const CChainParams& params) {
    if (!dest.IsValid()) return "";
    // version byte: type << 3 | size code (0 = 160 bits)
    std::vector<uint8_t> payload;
    payload.push_back((uint8_t)((dest.type == DestType::KEYID ? 0 : 1) << 3));
    payload.insert(payload.end(), dest.hash.begin(), dest.hash.end());
    std::vector<uint8_t> values;
    RegroupBits<8, 5, true>(values, payload.data(), payload.size());
    return cashaddr::Encode(params.CashAddrPrefix(), values);
}

CTxDestination DecodeCashAddr(const std::string& str, const CChainParams& params) {
    auto dec = cashaddr::Decode(str, params.CashAddrPrefix());
    if (dec.first != params.CashAddrPrefix() || dec.second.empty()) return CTxDestination();
    const std::vector<uint8_t>& values = dec.second;
    const size_t extrabits = values.size() * 5 % 8;
    if (extrabits >= 5) return CTxDestination();
    if (values.back() & ((1u << extrabits) - 1)) return CTxDestination();
    std::vector<uint8_t> data;
    RegroupBits<5, 8, true>(data, values.data(), values.size());
    // padding already validated; drop the trailing partial byte if any
    data.resize(values.size() * 5 / 8);
    if (data.empty()) return CTxDestination();
    const uint8_t version = data[0];
    if (version & 0x80) return CTxDestination();
    uint32_t hash_size = 20 + 4 * (version & 3);
    if (version & 4) hash_size *= 2;
    if (data.size() != hash_size + 1 || hash_size != 20) return CTxDestination();
    uint160 h;
    memcpy(h.begin(), data.data() + 1, 20);
    switch ((version >> 3) & 0x1f) {
    case 0: return CKeyID(h);
    case 1: return CScriptID(h);
    default: return CTxDestination();
    }
}

static std::atomic<bool> g_use_cashaddr{false}; // reference src/config.cpp:10 (GlobalConfig: useCashAddr(false))
void SetUseCashAddr(bool on) { g_use_cashaddr = on; }
bool UseCashAddr() { return g_use_cashaddr; }

std::string EncodeDestination(const CTxDestination& dest, const CChainParams& params) {
    return UseCashAddr() ? EncodeCashAddr(dest, params) : EncodeLegacyAddr(dest, params);
}
CTxDestination DecodeDestination(const std::string& str, const CChainParams& params) {
    CTxDestination d = DecodeCashAddr(str, params);
    if (d.IsValid()) return d;
    return DecodeLegacyAddr(str, params);
}
bool IsValidDestinationString(const std::string& str, const CChainParams& params) {
    return DecodeDestination(str, params).IsValid();
}

std::string EncodeSecret(const CKey& key, const CChainParams& params) {
    std::vector<unsigned char> d = params.Base58Prefix(CChainParams::SECRET_KEY);
    d.insert(d.end(), key.begin(), key.end());
    if (key.IsCompressed()) d.push_back(1);
    std::string s = EncodeBase58Check(d);
    memory_cleanse(d.data(), d.size());
    return s;
}
CKey DecodeSecret(const std::string& str, const CChainParams& params) {
    CKey key;
    std::vector<unsigned char> d;
    if (DecodeBase58Check(str, d)) {
        const auto& pre = params.Base58Prefix(CChainParams::SECRET_KEY);
        if ((d.size() == 32 + pre.size() || (d.size() == 33 + pre.size() && d.back() == 1)) &&
            std::equal(pre.begin(), pre.end(), d.begin())) {
            const bool compressed = d.size() == 33 + pre.size();
            key.Set(d.begin() + pre.size(), d.begin() + pre.size() + 32, compressed);
        }
    }
    if (!d.empty()) memory_cleanse(d.data(), d.size());
    return key;
}

template <typename K>
static std::string EncodeExt(const K& k, const std::vector<unsigned char>& pre) {
    std::vector<unsigned char> d = pre;
    const size_t n = d.size();
    d.resize(n + BIP32_EXTKEY_SIZE);
    k.Encode(d.data() + n);
    return EncodeBase58Check(d);
}
template <typename K>
static K DecodeExt(const std::string& str, const std::vector<unsigned char>& pre) {
    K k;
    std::vector<unsigned char> d;
    if (DecodeBase58Check(str, d) && d.size() == BIP32_EXTKEY_SIZE + pre.size() &&
        std::equal(pre.begin(), pre.end(), d.begin()))
        k.Decode(d.data() + pre.size());
    return k;
}
std::string EncodeExtKey(const CExtKey& key, const CChainParams& params) {
    return EncodeExt(key, params.Base58Prefix(CChainParams::EXT_SECRET_KEY));
}
CExtKey DecodeExtKey(const std::string& str, const CChainParams& params) {
    return DecodeExt<CExtKey>(str, params.Base58Prefix(CChainParams::EXT_SECRET_KEY));
}
std::string EncodeExtPubKey(const CExtPubKey& key, const CChainParams& params) {
    return EncodeExt(key, params.Base58Prefix(CChainParams::EXT_PUBLIC_KEY));
}
CExtPubKey DecodeExtPubKey(const std::string& str, const CChainParams& params) {
    return DecodeExt<CExtPubKey>(str, params.Base58Prefix(CChainParams::EXT_PUBLIC_KEY));
}

const std::string strMessageMagic = "Bitcoin Signed Message:\n";
uint256 MessageHash(const std::string& message) {
    HashWriter hw;
    hw << strMessageMagic << message;
    return hw.GetHash();
}

} // namespace bcp
