// Signature hash type wrapper (reference src/script/sighashtype.h:28): the base type (ALL /
// NONE / SINGLE in the low 5 bits) plus the FORKID (0x40) and ANYONECANPAY (0x80) flags, with
// copy-and-modify setters. The raw flag values are the interpreter's SIGHASH_* constants.
#pragma once
#include "script/interpreter.h"

#include <cstdint>
#include <stdexcept>

namespace bcp {

enum class BaseSigHashType : uint32_t { ALL = SIGHASH_ALL, NONE = SIGHASH_NONE, SINGLE = SIGHASH_SINGLE };

class SigHashType {
public:
    static constexpr uint32_t BASE_MASK = 0x1f;

    SigHashType() : raw(SIGHASH_ALL) {}
    // a raw value must name a base type (ALL, NONE or SINGLE)
    explicit SigHashType(uint32_t r) : raw(r) {
        const uint32_t base = raw & BASE_MASK;
        if (base < SIGHASH_ALL || base > SIGHASH_SINGLE) throw std::runtime_error("Base sighash must be specified");
    }

    SigHashType withBaseSigHash(BaseSigHashType b) const { return SigHashType((raw & ~BASE_MASK) | uint32_t(b)); }
    SigHashType withForkId(bool on) const { return SigHashType(Flag(SIGHASH_FORKID, on)); }
    SigHashType withAnyoneCanPay(bool on) const { return SigHashType(Flag(SIGHASH_ANYONECANPAY, on)); }

    BaseSigHashType getBaseSigHashType() const { return BaseSigHashType(raw & BASE_MASK); }
    bool hasForkId() const { return (raw & SIGHASH_FORKID) != 0; }
    bool hasAnyoneCanPay() const { return (raw & SIGHASH_ANYONECANPAY) != 0; }
    uint32_t getRawSigHashType() const { return raw; }

private:
    uint32_t Flag(uint32_t bit, bool on) const { return on ? (raw | bit) : (raw & ~bit); }
    uint32_t raw;
};

} // namespace bcp
