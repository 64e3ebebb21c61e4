#include "primitives/transaction.h"
#include "primitives/block.h"
#include "consensus/params.h"
#include "util/strencodings.h"

namespace bcp {

std::string COutPoint::ToString() const { return strprintf("COutPoint(%s, %u)", hash.ToString().substr(0, 10).c_str(), n); }

std::string CTxIn::ToString() const {
    std::string str = "CTxIn(" + prevout.ToString();
    if (prevout.IsNull()) str += ", coinbase " + HexStr(scriptSig);
    else str += ", scriptSig=" + HexStr(scriptSig).substr(0, 24);
    if (nSequence != SEQUENCE_FINAL) str += strprintf(", nSequence=%u", nSequence);
    return str + ")";
}

std::string CTxOut::ToString() const {
    return strprintf("CTxOut(nValue=%s, scriptPubKey=%s)", FormatMoney(nValue).c_str(),
                     HexStr(scriptPubKey).substr(0, 30).c_str());
}

std::string CFeeRate::ToString() const { return FormatMoney(nSatoshisPerK) + " BCP/kB"; }

CMutableTransaction::CMutableTransaction() : nVersion(CTransaction::CURRENT_VERSION), nLockTime(0) {}
CMutableTransaction::CMutableTransaction(const CTransaction& tx)
    : nVersion(tx.nVersion), vin(tx.vin), vout(tx.vout), nLockTime(tx.nLockTime) {}

uint256 CMutableTransaction::GetId() const { return SerializeHash(*this, SER_GETHASH, 0); }

// The txid, and the serialized size as a by-product (the same bytes are hashed)
uint256 CTransaction::ComputeHash() const {
    HashWriter hw(SER_GETHASH, 0);
    hw << *this;
    nTotalSize = (uint32_t)hw.BytesWritten();
    return hw.GetHash();
}

CTransaction::CTransaction() : nVersion(CTransaction::CURRENT_VERSION), vin(), vout(), nLockTime(0), hash() {}
CTransaction::CTransaction(const CMutableTransaction& tx)
    : nVersion(tx.nVersion), vin(tx.vin), vout(tx.vout), nLockTime(tx.nLockTime), hash(ComputeHash()) {}
CTransaction::CTransaction(CMutableTransaction&& tx)
    : nVersion(tx.nVersion), vin(std::move(tx.vin)), vout(std::move(tx.vout)), nLockTime(tx.nLockTime),
      hash(ComputeHash()) {}

Amount CTransaction::GetValueOut() const {
    Amount nValueOut = 0;
    for (const auto& out : vout) {
        nValueOut += out.nValue;
        if (!MoneyRange(out.nValue) || !MoneyRange(nValueOut)) throw std::runtime_error("GetValueOut: value out of range");
    }
    return nValueOut;
}

unsigned int CTransaction::GetTotalSize() const {
    // every serialized transaction is at least 10 bytes: 0 means not computed (default-constructed)
    return nTotalSize ? nTotalSize : (unsigned int)GetSerializeSize(*this, PROTOCOL_VERSION);
}

unsigned int CTransaction::CalculateModifiedSize(unsigned int nTxSize) const {
    // Discount inputs' scriptSig prefix overhead (reference CTransaction::CalculateModifiedSize).
    if (nTxSize == 0) nTxSize = GetTotalSize();
    for (const auto& in : vin) {
        unsigned int offset = 41U + std::min(110U, (unsigned int)in.scriptSig.size());
        if (nTxSize > offset) nTxSize -= offset;
    }
    return nTxSize;
}

double CTransaction::ComputePriority(double dPriorityInputs, unsigned int nTxSize) const {
    nTxSize = CalculateModifiedSize(nTxSize);
    if (nTxSize == 0) return 0.0;
    return dPriorityInputs / nTxSize;
}

std::string CTransaction::ToString() const {
    std::string str = strprintf("CTransaction(txid=%s, ver=%d, vin.size=%u, vout.size=%u, nLockTime=%u)\n",
                                GetId().ToString().substr(0, 10).c_str(), nVersion, (unsigned)vin.size(),
                                (unsigned)vout.size(), nLockTime);
    for (const auto& in : vin) str += "    " + in.ToString() + "\n";
    for (const auto& out : vout) str += "    " + out.ToString() + "\n";
    return str;
}

PrecomputedTransactionData::PrecomputedTransactionData(const CTransaction& tx) {
    HashWriter ssp, sss, sso;
    for (const auto& in : tx.vin) {
        ssp << in.prevout;
        sss << in.nSequence;
    }
    for (const auto& out : tx.vout) sso << out;
    hashPrevouts = ssp.GetHash();
    hashSequence = sss.GetHash();
    hashOutputs = sso.GetHash();
}

// ---------------------------------------------------------------- block
uint256 CBlockHeader::GetHashLegacy() const {
    HashWriter w(SER_GETHASH, PROTOCOL_VERSION | SERIALIZE_BLOCK_LEGACY);
    w << *this;
    return w.GetHash();
}
uint256 CBlockHeader::GetHashNew() const {
    HashWriter w(SER_GETHASH, PROTOCOL_VERSION);
    w << *this;
    return w.GetHash();
}
uint256 CBlockHeader::GetHash(const Consensus::Params& params) const {
    return nHeight >= (uint32_t)params.BCPHeight ? GetHashNew() : GetHashLegacy();
}
uint256 CBlockHeader::GetHash() const { return GetHash(Params().GetConsensus()); }

std::vector<unsigned char> CBlockHeader::EquihashInput() const {
    std::vector<unsigned char> out;
    VectorWriter w(out);
    w << nVersion << hashPrevBlock << hashMerkleRoot << nHeight;
    for (int i = 0; i < 7; ++i) w << nReserved[i];
    w << nTime << nBits;
    return out;
}

std::string CBlock::ToString() const {
    std::string s = strprintf("CBlock(hash=%s, ver=0x%08x, hashPrevBlock=%s, hashMerkleRoot=%s, nHeight=%u, nTime=%u, "
                              "nBits=%08x, nNonce=%s, vtx=%u)\n",
                              GetHash().ToString().c_str(), nVersion, hashPrevBlock.ToString().c_str(),
                              hashMerkleRoot.ToString().c_str(), nHeight, nTime, nBits, nNonce.GetHex().c_str(),
                              (unsigned)vtx.size());
    for (const auto& tx : vtx) s += "  " + tx->ToString() + "\n";
    return s;
}

} // namespace bcp
