// Monetary amounts and fee rates. Parity: reference src/amount.h:16-135 (Amount,
// COIN, CENT, MAX_MONEY = 21M coins, MoneyRange, CFeeRate per kB).
#pragma once
#include <cstdint>
#include <string>

namespace bcp {

typedef int64_t Amount;
static const Amount COIN = 100000000;
static const Amount CENT = 1000000;
static const Amount SATOSHI = 1;
static const Amount MAX_MONEY = 21000000 * COIN;
inline bool MoneyRange(Amount v) { return v >= 0 && v <= MAX_MONEY; }

// Fee rate in satoshis per 1000 bytes.
class CFeeRate {
    Amount nSatoshisPerK = 0;
public:
    CFeeRate() {}
    explicit CFeeRate(Amount perK) : nSatoshisPerK(perK) {}
    CFeeRate(Amount nFeePaid, size_t nBytes) {
        nSatoshisPerK = nBytes > 0 ? nFeePaid * 1000 / (int64_t)nBytes : 0;
    }
    Amount GetFee(size_t nBytes) const {
        Amount fee = nSatoshisPerK * (int64_t)nBytes / 1000;
        if (fee == 0 && nBytes != 0) {
            if (nSatoshisPerK > 0) fee = 1;
            if (nSatoshisPerK < 0) fee = -1;
        }
        return fee;
    }
    Amount GetFeePerK() const { return GetFee(1000); }
    friend bool operator<(const CFeeRate& a, const CFeeRate& b) { return a.nSatoshisPerK < b.nSatoshisPerK; }
    friend bool operator>(const CFeeRate& a, const CFeeRate& b) { return a.nSatoshisPerK > b.nSatoshisPerK; }
    friend bool operator==(const CFeeRate& a, const CFeeRate& b) { return a.nSatoshisPerK == b.nSatoshisPerK; }
    friend bool operator<=(const CFeeRate& a, const CFeeRate& b) { return a.nSatoshisPerK <= b.nSatoshisPerK; }
    friend bool operator>=(const CFeeRate& a, const CFeeRate& b) { return a.nSatoshisPerK >= b.nSatoshisPerK; }
    CFeeRate& operator+=(const CFeeRate& a) { nSatoshisPerK += a.nSatoshisPerK; return *this; }
    std::string ToString() const;
    template <typename S> void Serialize(S& s) const { s.write((const char*)&nSatoshisPerK, 8); }
    template <typename S> void Unserialize(S& s) { s.read((char*)&nSatoshisPerK, 8); }
};

} // namespace bcp
