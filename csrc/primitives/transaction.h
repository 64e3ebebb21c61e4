// Transactions. Wire format parity: reference src/primitives/transaction.{h,cpp}
// (COutPoint, CTxIn with sequence-lock flags, CTxOut, CTransaction with cached txid,
// CMutableTransaction, ComputeHash = SHA256d of the serialization).
#pragma once
#include "primitives/amount.h"
#include "primitives/serialize.h"
#include "primitives/uint256.h"
#include "script/script.h"

#include <memory>
#include <string>
#include <vector>

namespace bcp {

class COutPoint {
public:
    uint256 hash;
    uint32_t n = (uint32_t)-1;
    COutPoint() {}
    COutPoint(const uint256& h, uint32_t nIn) : hash(h), n(nIn) {}
    void SetNull() { hash.SetNull(); n = (uint32_t)-1; }
    bool IsNull() const { return hash.IsNull() && n == (uint32_t)-1; }
    friend bool operator<(const COutPoint& a, const COutPoint& b) {
        int c = a.hash.Compare(b.hash);
        return c < 0 || (c == 0 && a.n < b.n);
    }
    friend bool operator==(const COutPoint& a, const COutPoint& b) { return a.hash == b.hash && a.n == b.n; }
    friend bool operator!=(const COutPoint& a, const COutPoint& b) { return !(a == b); }
    std::string ToString() const;
    template <typename S> void Serialize(S& s) const { ::bcp::Serialize(s, hash); ::bcp::Serialize(s, n); }
    template <typename S> void Unserialize(S& s) { ::bcp::Unserialize(s, hash); ::bcp::Unserialize(s, n); }
};

struct OutPointHasher {
    size_t operator()(const COutPoint& o) const { return (size_t)(o.hash.GetCheapHash() ^ ((uint64_t)o.n * 0x9e3779b97f4a7c15ULL)); }
};

class CTxIn {
public:
    COutPoint prevout;
    CScript scriptSig;
    uint32_t nSequence = SEQUENCE_FINAL;

    static const uint32_t SEQUENCE_FINAL = 0xffffffff;
    static const uint32_t SEQUENCE_LOCKTIME_DISABLE_FLAG = (1U << 31);
    static const uint32_t SEQUENCE_LOCKTIME_TYPE_FLAG = (1 << 22);
    static const uint32_t SEQUENCE_LOCKTIME_MASK = 0x0000ffff;
    static const int SEQUENCE_LOCKTIME_GRANULARITY = 9;

    CTxIn() {}
    explicit CTxIn(COutPoint prevoutIn, CScript scriptSigIn = CScript(), uint32_t nSequenceIn = SEQUENCE_FINAL)
        : prevout(prevoutIn), scriptSig(scriptSigIn), nSequence(nSequenceIn) {}
    friend bool operator==(const CTxIn& a, const CTxIn& b) {
        return a.prevout == b.prevout && a.scriptSig == b.scriptSig && a.nSequence == b.nSequence;
    }
    std::string ToString() const;
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, prevout);
        ::bcp::Serialize(s, scriptSig);
        ::bcp::Serialize(s, nSequence);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, prevout);
        ::bcp::Unserialize(s, scriptSig);
        ::bcp::Unserialize(s, nSequence);
    }
};

class CTxOut {
public:
    Amount nValue = -1;
    CScript scriptPubKey;
    CTxOut() {}
    CTxOut(Amount v, CScript spk) : nValue(v), scriptPubKey(spk) {}
    void SetNull() { nValue = -1; scriptPubKey.clear(); }
    bool IsNull() const { return nValue == -1; }
    friend bool operator==(const CTxOut& a, const CTxOut& b) { return a.nValue == b.nValue && a.scriptPubKey == b.scriptPubKey; }
    friend bool operator!=(const CTxOut& a, const CTxOut& b) { return !(a == b); }
    std::string ToString() const;
    template <typename S> void Serialize(S& s) const { ::bcp::Serialize(s, nValue); ::bcp::Serialize(s, scriptPubKey); }
    template <typename S> void Unserialize(S& s) { ::bcp::Unserialize(s, nValue); ::bcp::Unserialize(s, scriptPubKey); }
};

class CMutableTransaction;

class CTransaction {
public:
    static const int32_t CURRENT_VERSION = 2;
    static const int32_t MAX_STANDARD_VERSION = 2;

    const int32_t nVersion;
    const std::vector<CTxIn> vin;
    const std::vector<CTxOut> vout;
    const uint32_t nLockTime;

    CTransaction();
    explicit CTransaction(const CMutableTransaction& tx);
    explicit CTransaction(CMutableTransaction&& tx);
    template <typename S> CTransaction(deserialize_type, S& s);

    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, vin);
        ::bcp::Serialize(s, vout);
        ::bcp::Serialize(s, nLockTime);
    }

    bool IsNull() const { return vin.empty() && vout.empty(); }
    const uint256& GetId() const { return hash; }
    const uint256& GetHash() const { return hash; }
    Amount GetValueOut() const;
    double ComputePriority(double dPriorityInputs, unsigned int nTxSize = 0) const;
    unsigned int CalculateModifiedSize(unsigned int nTxSize = 0) const;
    unsigned int GetTotalSize() const;
    bool IsCoinBase() const { return vin.size() == 1 && vin[0].prevout.IsNull(); }
    friend bool operator==(const CTransaction& a, const CTransaction& b) { return a.hash == b.hash; }
    friend bool operator!=(const CTransaction& a, const CTransaction& b) { return a.hash != b.hash; }
    std::string ToString() const;

private:
    mutable uint32_t nTotalSize = 0; // set by ComputeHash; declared before hash, so initialised first
    const uint256 hash;
    uint256 ComputeHash() const;
};

class CMutableTransaction {
public:
    int32_t nVersion;
    std::vector<CTxIn> vin;
    std::vector<CTxOut> vout;
    uint32_t nLockTime;

    CMutableTransaction();
    explicit CMutableTransaction(const CTransaction& tx);
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, vin);
        ::bcp::Serialize(s, vout);
        ::bcp::Serialize(s, nLockTime);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, nVersion);
        vin.clear();
        vout.clear();
        ::bcp::Unserialize(s, vin);
        ::bcp::Unserialize(s, vout);
        ::bcp::Unserialize(s, nLockTime);
    }
    uint256 GetId() const;
    friend bool operator==(const CMutableTransaction& a, const CMutableTransaction& b) { return a.GetId() == b.GetId(); }
};

template <typename S> CTransaction::CTransaction(deserialize_type, S& s) : CTransaction([&] {
    CMutableTransaction m;
    m.Unserialize(s);
    return m;
}()) {}

typedef std::shared_ptr<const CTransaction> CTransactionRef;
static inline CTransactionRef MakeTransactionRef() { return std::make_shared<const CTransaction>(); }
template <typename Tx> static inline CTransactionRef MakeTransactionRef(Tx&& txIn) {
    return std::make_shared<const CTransaction>(std::forward<Tx>(txIn));
}

// Per-transaction hashes reused by every input's FORKID signature digest
// (reference src/primitives/transaction.h:388 PrecomputedTransactionData).
struct PrecomputedTransactionData {
    uint256 hashPrevouts, hashSequence, hashOutputs;
    PrecomputedTransactionData() {}
    explicit PrecomputedTransactionData(const CTransaction& tx);
};

} // namespace bcp
