// BIP70 payment protocol: PaymentRequest / PaymentDetails / Payment / PaymentACK messages,
// certificate-chain merchant authentication and the request checks the wallet applies
// before paying.
//
// Parity: reference src/qt/paymentrequest.proto (message layout), src/qt/paymentrequestplus.cpp
// (parse :26-49, getMerchant :59-220, getPayTo :222-232) and the verify helpers of
// src/qt/paymentserver.cpp:844-890 (verifyNetwork, verifyExpired, verifySize, verifyAmount;
// BIP70_MAX_PAYMENTREQUEST_SIZE = 50000, paymentserver.h:52). The reference compiles the
// .proto with protoc and hangs the flow off Qt; here the proto2 wire format is encoded and
// decoded directly (no libprotobuf), and the flow is exposed through RPC
// (decodepaymentrequest / sendpaymentrequest) and the browser GUI instead of a Qt dialog.
#pragma once

#include "primitives/amount.h"
#include "script/script.h"

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace bcp {
namespace payments {

static const int64_t BIP70_MAX_PAYMENTREQUEST_SIZE = 50000;
static const char* const BIP71_MIMETYPE_PAYMENT = "application/bitcoincash-payment";
static const char* const BIP71_MIMETYPE_PAYMENTACK = "application/bitcoincash-paymentack";
static const char* const BIP71_MIMETYPE_PAYMENTREQUEST = "application/bitcoincash-paymentrequest";
static const bool DEFAULT_SELFSIGNED_ROOTCERTS = false;

// A field number + wire type + raw payload of a field this code does not know. proto2 keeps
// such fields and writes them back after the known ones, so a re-serialized request (the
// bytes a signature covers) matches what the merchant signed.
struct UnknownField {
    uint32_t key = 0;
    std::string raw; // encoded value (varint bytes, fixed bytes, or length-prefixed payload)
};

struct Output {
    uint64_t amount = 0;
    bool has_amount = false;
    std::string script;
    bool has_script = false;
    std::vector<UnknownField> unknown;
};

struct PaymentDetails {
    std::string network = "main";
    bool has_network = false;
    std::vector<Output> outputs;
    uint64_t time = 0;
    bool has_time = false;
    uint64_t expires = 0;
    bool has_expires = false;
    std::string memo, payment_url, merchant_data;
    bool has_memo = false, has_payment_url = false, has_merchant_data = false;
    std::vector<UnknownField> unknown;
};

struct PaymentRequest {
    uint32_t payment_details_version = 1;
    bool has_version = false;
    std::string pki_type = "none";
    bool has_pki_type = false;
    std::string pki_data;
    bool has_pki_data = false;
    std::string serialized_payment_details;
    bool has_details = false;
    std::string signature;
    bool has_signature = false;
    std::vector<UnknownField> unknown;
};

struct Payment {
    std::string merchant_data;
    bool has_merchant_data = false;
    std::vector<std::string> transactions;
    std::vector<Output> refund_to;
    std::string memo;
    bool has_memo = false;
};

struct PaymentACK {
    Payment payment;
    std::string memo;
    bool has_memo = false;
};

// proto2 encode/decode. Decoders return false on malformed input or a missing required field
// (ParseFromArray semantics).
bool ParseOutput(const std::string& in, Output& out);
bool ParsePaymentDetails(const std::string& in, PaymentDetails& out);
bool ParsePaymentRequest(const std::string& in, PaymentRequest& out);
bool ParseX509Certificates(const std::string& in, std::vector<std::string>& certs);
bool ParsePayment(const std::string& in, Payment& out);
bool ParsePaymentACK(const std::string& in, PaymentACK& out);
std::string SerializeOutput(const Output& o);
std::string SerializePaymentDetails(const PaymentDetails& d);
std::string SerializePaymentRequest(const PaymentRequest& r);
std::string SerializeX509Certificates(const std::vector<std::string>& certs);
std::string SerializePayment(const Payment& p);
std::string SerializePaymentACK(const PaymentACK& a);

// Trusted roots for merchant authentication: DER certificates, plus (optionally) the system
// store. `now` = 0 verifies at the current time.
struct CertStore {
    std::vector<std::string> roots_der;
    bool use_system = false;
    bool allow_self_signed_root = DEFAULT_SELFSIGNED_ROOTCERTS;
    int64_t now = 0;
};

// Loads -rootcertificates: "-system-" (the default) selects the system store, "" none, anything
// else is a PEM or DER file of root certificates. Returns false if the file cannot be read.
bool LoadRootCertificates(const std::string& setting, CertStore& store, std::string& err);

class PaymentRequestPlus {
public:
    bool parse(const std::string& data);
    bool IsInitialized() const { return initialized; }
    // Verified merchant name (subject common name of the signing certificate), or false with
    // `err` set: pki_type none/unknown, bad chain, expired certificate, untrusted root, bad
    // signature or a certificate without a common name.
    bool getMerchant(const CertStore& store, std::string& merchant, std::string* err = nullptr) const;
    std::vector<std::pair<CScript, Amount>> getPayTo() const;
    const PaymentDetails& getDetails() const { return details; }
    const PaymentRequest& getRequest() const { return request; }
    std::string SerializeToString() const { return SerializePaymentRequest(request); }

private:
    PaymentRequest request;
    PaymentDetails details;
    bool initialized = false;
};

bool VerifyNetwork(const PaymentDetails& d, const std::string& networkId);
bool VerifyExpired(const PaymentDetails& d, int64_t now); // true = expired
bool VerifySize(int64_t size);
bool VerifyAmount(Amount a);

} // namespace payments
} // namespace bcp
