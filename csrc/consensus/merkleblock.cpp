#include "consensus/merkleblock.h"
#include "crypto/common.h"
#include "keys/key.h"
#include "script/standard.h"

#include <cmath>

namespace bcp {

static inline uint32_t ROTL32(uint32_t x, int8_t r) { return (x << r) | (x >> (32 - r)); }

// MurmurHash3 x86_32 (public-domain algorithm by Austin Appleby).
uint32_t MurmurHash3(uint32_t nHashSeed, const unsigned char* data, size_t len) {
    uint32_t h1 = nHashSeed;
    const uint32_t c1 = 0xcc9e2d51, c2 = 0x1b873593;
    const size_t nblocks = len / 4;
    for (size_t i = 0; i < nblocks; ++i) {
        uint32_t k1 = ReadLE32(data + i * 4);
        k1 *= c1;
        k1 = ROTL32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
        h1 = ROTL32(h1, 13);
        h1 = h1 * 5 + 0xe6546b64;
    }
    const unsigned char* tail = data + nblocks * 4;
    uint32_t k1 = 0;
    switch (len & 3) {
    case 3: k1 ^= tail[2] << 16; // fallthrough
    case 2: k1 ^= tail[1] << 8;  // fallthrough
    case 1:
        k1 ^= tail[0];
        k1 *= c1;
        k1 = ROTL32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16;
    h1 *= 0x85ebca6b;
    h1 ^= h1 >> 13;
    h1 *= 0xc2b2ae35;
    h1 ^= h1 >> 16;
    return h1;
}

// ------------------------------------------------------------------ CBloomFilter
#define LN2SQUARED 0.4804530139182014246671025263266649717305529515945455
#define LN2 0.6931471805599453094172321214581765680755001343602552

CBloomFilter::CBloomFilter(unsigned nElements, double nFPRate, unsigned nTweakIn, unsigned char nFlagsIn)
    : vData(std::min((unsigned)(-1 / LN2SQUARED * nElements * std::log(nFPRate)), MAX_BLOOM_FILTER_SIZE * 8) / 8),
      isFull(false), isEmpty(true),
      nHashFuncs(std::min((unsigned)(vData.size() * 8 / std::max(1u, nElements) * LN2), MAX_HASH_FUNCS)),
      nTweak(nTweakIn), nFlags(nFlagsIn) {}

unsigned CBloomFilter::Hash(unsigned nHashNum, const std::vector<unsigned char>& d) const {
    return MurmurHash3(nHashNum * 0xFBA4C795 + nTweak, d.data(), d.size()) % (vData.size() * 8);
}
void CBloomFilter::insert(const std::vector<unsigned char>& vKey) {
    if (isFull || vData.empty()) return;
    for (unsigned i = 0; i < nHashFuncs; i++) {
        const unsigned nIndex = Hash(i, vKey);
        vData[nIndex >> 3] |= (1 << (7 & nIndex));
    }
    isEmpty = false;
}
void CBloomFilter::insert(const COutPoint& outpoint) { insert(SerializeToBytes(outpoint)); }
void CBloomFilter::insert(const uint256& hash) { insert(std::vector<unsigned char>(hash.begin(), hash.end())); }
bool CBloomFilter::contains(const std::vector<unsigned char>& vKey) const {
    if (isFull) return true;
    if (isEmpty || vData.empty()) return false;
    for (unsigned i = 0; i < nHashFuncs; i++) {
        const unsigned nIndex = Hash(i, vKey);
        if (!(vData[nIndex >> 3] & (1 << (7 & nIndex)))) return false;
    }
    return true;
}
bool CBloomFilter::contains(const COutPoint& outpoint) const { return contains(SerializeToBytes(outpoint)); }
bool CBloomFilter::contains(const uint256& hash) const { return contains(std::vector<unsigned char>(hash.begin(), hash.end())); }
void CBloomFilter::clear() {
    vData.assign(vData.size(), 0);
    isFull = false;
    isEmpty = true;
}
void CBloomFilter::reset(unsigned nNewTweak) {
    clear();
    nTweak = nNewTweak;
}
bool CBloomFilter::IsWithinSizeConstraints() const {
    return vData.size() <= MAX_BLOOM_FILTER_SIZE && nHashFuncs <= MAX_HASH_FUNCS;
}
void CBloomFilter::UpdateEmptyFull() {
    bool full = true, empty = true;
    for (unsigned char c : vData) {
        full &= c == 0xff;
        empty &= c == 0;
    }
    isFull = full;
    isEmpty = empty;
}
bool CBloomFilter::IsRelevantAndUpdate(const CTransaction& tx) {
    bool fFound = false;
    if (isFull) return true;
    if (isEmpty) return false;
    const uint256& hash = tx.GetHash();
    if (contains(hash)) fFound = true;
    for (unsigned i = 0; i < tx.vout.size(); i++) {
        const CTxOut& txout = tx.vout[i];
        CScript::const_iterator pc = txout.scriptPubKey.begin();
        std::vector<unsigned char> data;
        while (pc < txout.scriptPubKey.end()) {
            opcodetype opcode;
            if (!txout.scriptPubKey.GetOp(pc, opcode, data)) break;
            if (data.size() != 0 && contains(data)) {
                fFound = true;
                if ((nFlags & BLOOM_UPDATE_MASK) == BLOOM_UPDATE_ALL) {
                    insert(COutPoint(hash, i));
                } else if ((nFlags & BLOOM_UPDATE_MASK) == BLOOM_UPDATE_P2PUBKEY_ONLY) {
                    txnouttype type;
                    std::vector<std::vector<unsigned char>> sol;
                    if (Solver(txout.scriptPubKey, type, sol) && (type == TX_PUBKEY || type == TX_MULTISIG))
                        insert(COutPoint(hash, i));
                }
                break;
            }
        }
    }
    if (fFound) return true;
    for (const CTxIn& txin : tx.vin) {
        if (contains(txin.prevout)) return true;
        CScript::const_iterator pc = txin.scriptSig.begin();
        std::vector<unsigned char> data;
        while (pc < txin.scriptSig.end()) {
            opcodetype opcode;
            if (!txin.scriptSig.GetOp(pc, opcode, data)) break;
            if (data.size() != 0 && contains(data)) return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------ CRollingBloomFilter
// Three generations encoded in two bit-planes; each insert stamps the current
// generation, advancing a generation clears the oldest one.
CRollingBloomFilter::CRollingBloomFilter(unsigned nElements, double fpRate) {
    const double logFpRate = std::log(fpRate);
    nHashFuncs = std::max(1, std::min((int)std::round(logFpRate / std::log(0.5)), 50));
    nEntriesPerGeneration = (int)((nElements + 1) / 2);
    const uint32_t nMaxElements = nEntriesPerGeneration * 3;
    const uint32_t nFilterBits =
        (uint32_t)std::ceil(-1.0 * nHashFuncs * nMaxElements / std::log(1.0 - std::exp(logFpRate / nHashFuncs)));
    data.assign(((nFilterBits + 63) / 64) << 1, 0);
    reset();
}
static inline uint32_t RollingBloomHash(unsigned n, unsigned tweak, const std::vector<unsigned char>& v) {
    return MurmurHash3(n * 0xFBA4C795 + tweak, v.data(), v.size());
}
void CRollingBloomFilter::insert(const std::vector<unsigned char>& vKey) {
    if (nEntriesThisGeneration == nEntriesPerGeneration) {
        nEntriesThisGeneration = 0;
        nGeneration++;
        if (nGeneration == 4) nGeneration = 1;
        const uint64_t m1 = 0 - (uint64_t)(nGeneration & 1), m2 = 0 - (uint64_t)(nGeneration >> 1);
        for (size_t p = 0; p < data.size(); p += 2) {
            const uint64_t p1 = data[p], p2 = data[p + 1];
            const uint64_t mask = (p1 ^ m1) | (p2 ^ m2);
            data[p] = p1 & mask;
            data[p + 1] = p2 & mask;
        }
    }
    nEntriesThisGeneration++;
    for (int n = 0; n < nHashFuncs; n++) {
        const uint32_t h = RollingBloomHash(n, nTweak, vKey);
        const int bit = h & 0x3F;
        const uint32_t pos = (h >> 6) % data.size();
        data[pos & ~1u] = (data[pos & ~1u] & ~(((uint64_t)1) << bit)) | ((uint64_t)(nGeneration & 1)) << bit;
        data[pos | 1] = (data[pos | 1] & ~(((uint64_t)1) << bit)) | ((uint64_t)(nGeneration >> 1)) << bit;
    }
}
void CRollingBloomFilter::insert(const uint256& hash) { insert(std::vector<unsigned char>(hash.begin(), hash.end())); }
bool CRollingBloomFilter::contains(const std::vector<unsigned char>& vKey) const {
    for (int n = 0; n < nHashFuncs; n++) {
        const uint32_t h = RollingBloomHash(n, nTweak, vKey);
        const int bit = h & 0x3F;
        const uint32_t pos = (h >> 6) % data.size();
        if (!(((data[pos & ~1u] | data[pos | 1]) >> bit) & 1)) return false;
    }
    return true;
}
bool CRollingBloomFilter::contains(const uint256& hash) const {
    return contains(std::vector<unsigned char>(hash.begin(), hash.end()));
}
void CRollingBloomFilter::reset() {
    nTweak = (unsigned)GetRand(0xFFFFFFFFu);
    nEntriesThisGeneration = 0;
    nGeneration = 1;
    std::fill(data.begin(), data.end(), 0);
}

// ------------------------------------------------------------------ partial merkle tree
CPartialMerkleTree::CPartialMerkleTree() {}

CPartialMerkleTree::CPartialMerkleTree(const std::vector<uint256>& vTxid, const std::vector<bool>& vMatch)
    : nTransactions((unsigned)vTxid.size()) {
    int nHeight = 0;
    while (CalcTreeWidth(nHeight) > 1) nHeight++;
    TraverseAndBuild(nHeight, 0, vTxid, vMatch);
}

uint256 CPartialMerkleTree::CalcHash(int height, unsigned pos, const std::vector<uint256>& vTxid) {
    if (height == 0) return vTxid[pos];
    const uint256 left = CalcHash(height - 1, pos * 2, vTxid);
    const uint256 right = pos * 2 + 1 < CalcTreeWidth(height - 1) ? CalcHash(height - 1, pos * 2 + 1, vTxid) : left;
    return Hash256Concat(left, right);
}

void CPartialMerkleTree::TraverseAndBuild(int height, unsigned pos, const std::vector<uint256>& vTxid,
                                          const std::vector<bool>& vMatch) {
    bool fParentOfMatch = false;
    for (unsigned p = pos << height; p < (pos + 1) << height && p < nTransactions; p++) fParentOfMatch |= vMatch[p];
    vBits.push_back(fParentOfMatch);
    if (height == 0 || !fParentOfMatch) {
        vHash.push_back(CalcHash(height, pos, vTxid));
    } else {
        TraverseAndBuild(height - 1, pos * 2, vTxid, vMatch);
        if (pos * 2 + 1 < CalcTreeWidth(height - 1)) TraverseAndBuild(height - 1, pos * 2 + 1, vTxid, vMatch);
    }
}

uint256 CPartialMerkleTree::TraverseAndExtract(int height, unsigned pos, unsigned& nBitsUsed, unsigned& nHashUsed,
                                               std::vector<uint256>& vMatch, std::vector<unsigned>& vnIndex) {
    if (nBitsUsed >= vBits.size()) {
        fBad = true;
        return uint256();
    }
    const bool fParentOfMatch = vBits[nBitsUsed++];
    if (height == 0 || !fParentOfMatch) {
        if (nHashUsed >= vHash.size()) {
            fBad = true;
            return uint256();
        }
        const uint256& hash = vHash[nHashUsed++];
        if (height == 0 && fParentOfMatch) {
            vMatch.push_back(hash);
            vnIndex.push_back(pos);
        }
        return hash;
    }
    const uint256 left = TraverseAndExtract(height - 1, pos * 2, nBitsUsed, nHashUsed, vMatch, vnIndex);
    uint256 right;
    if (pos * 2 + 1 < CalcTreeWidth(height - 1)) {
        right = TraverseAndExtract(height - 1, pos * 2 + 1, nBitsUsed, nHashUsed, vMatch, vnIndex);
        if (right == left) fBad = true; // CVE-2012-2459: identical siblings would allow fake txids
    } else {
        right = left;
    }
    return Hash256Concat(left, right);
}

uint256 CPartialMerkleTree::ExtractMatches(std::vector<uint256>& vMatch, std::vector<unsigned>& vnIndex) {
    vMatch.clear();
    if (nTransactions == 0) return uint256();
    if (nTransactions > 32 * 1000000 / 60) return uint256(); // more than a 32 MB block could hold
    if (vHash.size() > nTransactions) return uint256();
    if (vBits.size() < vHash.size()) return uint256();
    int nHeight = 0;
    while (CalcTreeWidth(nHeight) > 1) nHeight++;
    unsigned nBitsUsed = 0, nHashUsed = 0;
    const uint256 hashMerkleRoot = TraverseAndExtract(nHeight, 0, nBitsUsed, nHashUsed, vMatch, vnIndex);
    if (fBad) return uint256();
    if ((nBitsUsed + 7) / 8 != (vBits.size() + 7) / 8) return uint256();
    if (nHashUsed != vHash.size()) return uint256();
    return hashMerkleRoot;
}

CMerkleBlock::CMerkleBlock(const CBlock& block, CBloomFilter& filter) {
    header = block.GetBlockHeader();
    std::vector<bool> vMatch;
    std::vector<uint256> vHashes;
    for (unsigned i = 0; i < block.vtx.size(); i++) {
        const uint256& hash = block.vtx[i]->GetHash();
        if (filter.IsRelevantAndUpdate(*block.vtx[i])) {
            vMatch.push_back(true);
            vMatchedTxn.push_back(std::make_pair(i, hash));
        } else {
            vMatch.push_back(false);
        }
        vHashes.push_back(hash);
    }
    txn = CPartialMerkleTree(vHashes, vMatch);
}

CMerkleBlock::CMerkleBlock(const CBlock& block, const std::set<uint256>& txids) {
    header = block.GetBlockHeader();
    std::vector<bool> vMatch;
    std::vector<uint256> vHashes;
    for (const auto& tx : block.vtx) {
        vMatch.push_back(txids.count(tx->GetHash()) > 0);
        vHashes.push_back(tx->GetHash());
    }
    txn = CPartialMerkleTree(vHashes, vMatch);
}

bool DecodeTxOutProof(const std::vector<unsigned char>& data, CMerkleBlock& mb) {
    for (int legacy = 0; legacy < 2; legacy++) {
        try {
            SpanReader r(data.data(), data.size(), SER_NETWORK, PROTOCOL_VERSION | (legacy ? SERIALIZE_BLOCK_LEGACY : 0));
            r >> mb;
            if (r.empty()) return true;
        } catch (const std::exception&) {
        }
    }
    return false;
}

} // namespace bcp
