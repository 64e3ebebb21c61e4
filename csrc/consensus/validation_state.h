// Validation outcome with DoS score and reject code.
// Parity: reference src/consensus/validation.h (REJECT_* codes, CValidationState
// DoS/Invalid/Error modes, corruption flag).
#pragma once
#include <cstdint>
#include <string>

namespace bcp {

static const uint8_t REJECT_MALFORMED = 0x01;
static const uint8_t REJECT_INVALID = 0x10;
static const uint8_t REJECT_OBSOLETE = 0x11;
static const uint8_t REJECT_DUPLICATE = 0x12;
static const uint8_t REJECT_NONSTANDARD = 0x40;
static const uint8_t REJECT_DUST = 0x41;
static const uint8_t REJECT_INSUFFICIENTFEE = 0x42;
static const uint8_t REJECT_CHECKPOINT = 0x43;

class CValidationState {
public:
    bool DoS(int level, bool ret = false, unsigned code = 0, const std::string& reason = "", bool corruption = false,
             const std::string& debug = "") {
        chRejectCode = code;
        strRejectReason = reason;
        corruptionPossible = corruption;
        strDebugMessage = debug;
        if (mode == MODE_ERROR) return ret;
        nDoS += level;
        mode = MODE_INVALID;
        return ret;
    }
    bool Invalid(bool ret = false, unsigned code = 0, const std::string& reason = "", const std::string& debug = "") {
        return DoS(0, ret, code, reason, false, debug);
    }
    bool Error(const std::string& reason) {
        if (mode == MODE_VALID) strRejectReason = reason;
        mode = MODE_ERROR;
        return false;
    }
    bool IsValid() const { return mode == MODE_VALID; }
    bool IsInvalid() const { return mode == MODE_INVALID; }
    bool IsError() const { return mode == MODE_ERROR; }
    bool IsInvalid(int& nDoSOut) const {
        if (!IsInvalid()) return false;
        nDoSOut = nDoS;
        return true;
    }
    bool CorruptionPossible() const { return corruptionPossible; }
    void SetCorruptionPossible() { corruptionPossible = true; }
    unsigned GetRejectCode() const { return chRejectCode; }
    const std::string& GetRejectReason() const { return strRejectReason; }
    const std::string& GetDebugMessage() const { return strDebugMessage; }
    std::string ToString() const {
        return strRejectReason + (strDebugMessage.empty() ? "" : ", " + strDebugMessage) +
               (chRejectCode ? " (code " + std::to_string(chRejectCode) + ")" : "");
    }

private:
    enum { MODE_VALID, MODE_INVALID, MODE_ERROR } mode = MODE_VALID;
    int nDoS = 0;
    std::string strRejectReason;
    unsigned chRejectCode = 0;
    bool corruptionPossible = false;
    std::string strDebugMessage;
};

} // namespace bcp
