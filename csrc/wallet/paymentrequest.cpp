// BIP70 payment protocol codec and merchant authentication (see paymentrequest.h for parity).
#include "wallet/paymentrequest.h"

#include "util/util.h"

#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/x509.h>
#include <openssl/x509_vfy.h>

#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>

namespace bcp {
namespace payments {

namespace {

// ---------------------------------------------------------------- proto2 wire format
enum WireType { WT_VARINT = 0, WT_FIXED64 = 1, WT_LEN = 2, WT_FIXED32 = 5 };

class Reader {
public:
    explicit Reader(const std::string& s) : p((const unsigned char*)s.data()), end(p + s.size()) {}
    bool done() const { return p == end; }
    bool varint(uint64_t& v) {
        v = 0;
        for (int shift = 0; shift < 64; shift += 7) {
            if (p == end) return false;
            const unsigned char b = *p++;
            v |= (uint64_t)(b & 0x7f) << shift;
            if (!(b & 0x80)) return true;
        }
        return false; // more than 10 bytes
    }
    bool bytes(std::string& out) {
        uint64_t n;
        if (!varint(n) || n > (uint64_t)(end - p)) return false;
        out.assign((const char*)p, (size_t)n);
        p += n;
        return true;
    }
    // Skip a field's value, capturing its encoding (unknown-field preservation).
    bool skip(int wt, std::string& raw) {
        const unsigned char* s = p;
        uint64_t n;
        switch (wt) {
        case WT_VARINT:
            if (!varint(n)) return false;
            break;
        case WT_FIXED64:
            if (end - p < 8) return false;
            p += 8;
            break;
        case WT_FIXED32:
            if (end - p < 4) return false;
            p += 4;
            break;
        case WT_LEN:
            if (!varint(n) || n > (uint64_t)(end - p)) return false;
            p += n;
            break;
        default:
            return false; // groups (3/4) are not used by these messages
        }
        raw.assign((const char*)s, p - s);
        return true;
    }

private:
    const unsigned char* p;
    const unsigned char* end;
};

void PutVarint(std::string& o, uint64_t v) {
    while (v >= 0x80) {
        o.push_back((char)((v & 0x7f) | 0x80));
        v >>= 7;
    }
    o.push_back((char)v);
}
void PutKey(std::string& o, int field, int wt) { PutVarint(o, ((uint64_t)field << 3) | (uint64_t)wt); }
void PutBytes(std::string& o, int field, const std::string& s) {
    PutKey(o, field, WT_LEN);
    PutVarint(o, s.size());
    o += s;
}
void PutUint(std::string& o, int field, uint64_t v) {
    PutKey(o, field, WT_VARINT);
    PutVarint(o, v);
}
void PutUnknown(std::string& o, const std::vector<UnknownField>& u) {
    for (const auto& f : u) {
        PutVarint(o, f.key);
        o += f.raw;
    }
}

// Generic field loop: `known(field, wt, reader)` returns 1 handled, 0 unknown, -1 error.
template <class F> bool ParseFields(const std::string& in, std::vector<UnknownField>* unknown, F known) {
    Reader r(in);
    while (!r.done()) {
        uint64_t key;
        if (!r.varint(key) || key > 0xffffffffu) return false;
        const int field = (int)(key >> 3), wt = (int)(key & 7);
        if (field == 0) return false;
        const int k = known(field, wt, r);
        if (k < 0) return false;
        if (k == 0) {
            UnknownField u;
            u.key = (uint32_t)key;
            if (!r.skip(wt, u.raw)) return false;
            if (unknown) unknown->push_back(std::move(u));
        }
    }
    return true;
}

struct X509Deleter {
    void operator()(X509* x) const { X509_free(x); }
};
struct StoreDeleter {
    void operator()(X509_STORE* s) const { X509_STORE_free(s); }
};
struct CtxDeleter {
    void operator()(X509_STORE_CTX* c) const { X509_STORE_CTX_free(c); }
};
struct MdCtxDeleter {
    void operator()(EVP_MD_CTX* c) const { EVP_MD_CTX_free(c); }
};
struct PkeyDeleter {
    void operator()(EVP_PKEY* k) const { EVP_PKEY_free(k); }
};

X509* DecodeDer(const std::string& der) {
    const unsigned char* d = (const unsigned char*)der.data();
    return d2i_X509(nullptr, &d, (long)der.size());
}

} // namespace

// ---------------------------------------------------------------- messages
bool ParseOutput(const std::string& in, Output& o) {
    o = Output();
    const bool ok = ParseFields(in, &o.unknown, [&](int f, int wt, Reader& r) -> int {
        if (f == 1 && wt == WT_VARINT) return r.varint(o.amount) ? (o.has_amount = true, 1) : -1;
        if (f == 2 && wt == WT_LEN) return r.bytes(o.script) ? (o.has_script = true, 1) : -1;
        return 0;
    });
    return ok && o.has_script;
}

std::string SerializeOutput(const Output& o) {
    std::string s;
    if (o.has_amount) PutUint(s, 1, o.amount);
    if (o.has_script) PutBytes(s, 2, o.script);
    PutUnknown(s, o.unknown);
    return s;
}

bool ParsePaymentDetails(const std::string& in, PaymentDetails& d) {
    d = PaymentDetails();
    const bool ok = ParseFields(in, &d.unknown, [&](int f, int wt, Reader& r) -> int {
        std::string b;
        switch (f) {
        case 1:
            if (wt != WT_LEN) return 0;
            return r.bytes(d.network) ? (d.has_network = true, 1) : -1;
        case 2: {
            if (wt != WT_LEN) return 0;
            Output o;
            if (!r.bytes(b) || !ParseOutput(b, o)) return -1;
            d.outputs.push_back(std::move(o));
            return 1;
        }
        case 3:
            if (wt != WT_VARINT) return 0;
            return r.varint(d.time) ? (d.has_time = true, 1) : -1;
        case 4:
            if (wt != WT_VARINT) return 0;
            return r.varint(d.expires) ? (d.has_expires = true, 1) : -1;
        case 5:
            if (wt != WT_LEN) return 0;
            return r.bytes(d.memo) ? (d.has_memo = true, 1) : -1;
        case 6:
            if (wt != WT_LEN) return 0;
            return r.bytes(d.payment_url) ? (d.has_payment_url = true, 1) : -1;
        case 7:
            if (wt != WT_LEN) return 0;
            return r.bytes(d.merchant_data) ? (d.has_merchant_data = true, 1) : -1;
        }
        return 0;
    });
    return ok && d.has_time;
}

std::string SerializePaymentDetails(const PaymentDetails& d) {
    std::string s;
    if (d.has_network) PutBytes(s, 1, d.network);
    for (const auto& o : d.outputs) PutBytes(s, 2, SerializeOutput(o));
    if (d.has_time) PutUint(s, 3, d.time);
    if (d.has_expires) PutUint(s, 4, d.expires);
    if (d.has_memo) PutBytes(s, 5, d.memo);
    if (d.has_payment_url) PutBytes(s, 6, d.payment_url);
    if (d.has_merchant_data) PutBytes(s, 7, d.merchant_data);
    PutUnknown(s, d.unknown);
    return s;
}

bool ParsePaymentRequest(const std::string& in, PaymentRequest& q) {
    q = PaymentRequest();
    const bool ok = ParseFields(in, &q.unknown, [&](int f, int wt, Reader& r) -> int {
        uint64_t v;
        switch (f) {
        case 1:
            if (wt != WT_VARINT) return 0;
            if (!r.varint(v)) return -1;
            q.payment_details_version = (uint32_t)v; // uint32 field: truncating, as protobuf does
            q.has_version = true;
            return 1;
        case 2:
            if (wt != WT_LEN) return 0;
            return r.bytes(q.pki_type) ? (q.has_pki_type = true, 1) : -1;
        case 3:
            if (wt != WT_LEN) return 0;
            return r.bytes(q.pki_data) ? (q.has_pki_data = true, 1) : -1;
        case 4:
            if (wt != WT_LEN) return 0;
            return r.bytes(q.serialized_payment_details) ? (q.has_details = true, 1) : -1;
        case 5:
            if (wt != WT_LEN) return 0;
            return r.bytes(q.signature) ? (q.has_signature = true, 1) : -1;
        }
        return 0;
    });
    return ok && q.has_details;
}

std::string SerializePaymentRequest(const PaymentRequest& q) {
    std::string s;
    if (q.has_version) PutUint(s, 1, q.payment_details_version);
    if (q.has_pki_type) PutBytes(s, 2, q.pki_type);
    if (q.has_pki_data) PutBytes(s, 3, q.pki_data);
    if (q.has_details) PutBytes(s, 4, q.serialized_payment_details);
    if (q.has_signature) PutBytes(s, 5, q.signature);
    PutUnknown(s, q.unknown);
    return s;
}

bool ParseX509Certificates(const std::string& in, std::vector<std::string>& certs) {
    certs.clear();
    return ParseFields(in, nullptr, [&](int f, int wt, Reader& r) -> int {
        if (f != 1 || wt != WT_LEN) return 0;
        std::string c;
        if (!r.bytes(c)) return -1;
        certs.push_back(std::move(c));
        return 1;
    });
}

std::string SerializeX509Certificates(const std::vector<std::string>& certs) {
    std::string s;
    for (const auto& c : certs) PutBytes(s, 1, c);
    return s;
}

bool ParsePayment(const std::string& in, Payment& p) {
    p = Payment();
    return ParseFields(in, nullptr, [&](int f, int wt, Reader& r) -> int {
        if (wt != WT_LEN) return 0;
        std::string b;
        switch (f) {
        case 1:
            return r.bytes(p.merchant_data) ? (p.has_merchant_data = true, 1) : -1;
        case 2:
            if (!r.bytes(b)) return -1;
            p.transactions.push_back(std::move(b));
            return 1;
        case 3: {
            Output o;
            if (!r.bytes(b) || !ParseOutput(b, o)) return -1;
            p.refund_to.push_back(std::move(o));
            return 1;
        }
        case 4:
            return r.bytes(p.memo) ? (p.has_memo = true, 1) : -1;
        }
        return 0;
    });
}

std::string SerializePayment(const Payment& p) {
    std::string s;
    if (p.has_merchant_data) PutBytes(s, 1, p.merchant_data);
    for (const auto& t : p.transactions) PutBytes(s, 2, t);
    for (const auto& o : p.refund_to) PutBytes(s, 3, SerializeOutput(o));
    if (p.has_memo) PutBytes(s, 4, p.memo);
    return s;
}

bool ParsePaymentACK(const std::string& in, PaymentACK& a) {
    a = PaymentACK();
    bool has_payment = false;
    const bool ok = ParseFields(in, nullptr, [&](int f, int wt, Reader& r) -> int {
        if (wt != WT_LEN) return 0;
        std::string b;
        if (f == 1) {
            // a repeated embedded message merges; one Payment per ACK is all BIP70 sends
            if (!r.bytes(b) || !ParsePayment(b, a.payment)) return -1;
            has_payment = true;
            return 1;
        }
        if (f == 2) return r.bytes(a.memo) ? (a.has_memo = true, 1) : -1;
        return 0;
    });
    return ok && has_payment;
}

std::string SerializePaymentACK(const PaymentACK& a) {
    std::string s;
    PutBytes(s, 1, SerializePayment(a.payment));
    if (a.has_memo) PutBytes(s, 2, a.memo);
    return s;
}

// ---------------------------------------------------------------- root certificates
bool LoadRootCertificates(const std::string& setting, CertStore& store, std::string& err) {
    store.roots_der.clear();
    store.use_system = false;
    if (setting == "-system-") {
        store.use_system = true;
        return true;
    }
    if (setting.empty()) return true;
    std::ifstream f(setting, std::ios::binary);
    if (!f) {
        err = "cannot read root certificate file " + setting;
        return false;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string data = ss.str();
    if (data.find("-----BEGIN CERTIFICATE-----") != std::string::npos) {
        BIO* bio = BIO_new_mem_buf(data.data(), (int)data.size());
        for (;;) {
            X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
            if (!x) break;
            unsigned char* der = nullptr;
            const int n = i2d_X509(x, &der);
            if (n > 0) store.roots_der.emplace_back((const char*)der, (size_t)n);
            OPENSSL_free(der);
            X509_free(x);
        }
        BIO_free(bio);
    } else if (std::unique_ptr<X509, X509Deleter> x{DecodeDer(data)}) {
        store.roots_der.push_back(data);
    }
    if (store.roots_der.empty()) {
        err = "no certificates in " + setting;
        return false;
    }
    return true;
}

// ---------------------------------------------------------------- PaymentRequestPlus
bool PaymentRequestPlus::parse(const std::string& data) {
    initialized = false;
    details = PaymentDetails();
    if (!ParsePaymentRequest(data, request)) {
        LogPrintf("PaymentRequestPlus::parse: Error parsing payment request\n");
        request = PaymentRequest();
        return false;
    }
    if (request.payment_details_version > 1) {
        LogPrintf("PaymentRequestPlus::parse: Received up-version payment details, version=%u\n",
                  request.payment_details_version);
        return false;
    }
    if (!ParsePaymentDetails(request.serialized_payment_details, details)) {
        LogPrintf("PaymentRequestPlus::parse: Error parsing payment details\n");
        request = PaymentRequest();
        details = PaymentDetails();
        return false;
    }
    initialized = true;
    return true;
}

bool PaymentRequestPlus::getMerchant(const CertStore& cs, std::string& merchant, std::string* err) const {
    merchant.clear();
    auto fail = [&](const std::string& e) {
        if (err) *err = e;
        LogPrintf("PaymentRequestPlus::getMerchant: %s\n", e.c_str());
        return false;
    };
    if (!initialized) return fail("payment request not initialized");
    const EVP_MD* md = nullptr;
    if (request.pki_type == "x509+sha256") md = EVP_sha256();
    else if (request.pki_type == "x509+sha1") md = EVP_sha1();
    else if (request.pki_type == "none") return fail("pki_type == none");
    else return fail("unknown pki_type " + request.pki_type);

    std::vector<std::string> ders;
    if (!ParseX509Certificates(request.pki_data, ders)) return fail("error parsing pki_data");
    std::vector<std::unique_ptr<X509, X509Deleter>> certs;
    for (const auto& d : ders)
        if (X509* x = DecodeDer(d)) certs.emplace_back(x);
    if (certs.empty()) return fail("empty certificate chain");

    time_t now = cs.now ? (time_t)cs.now : (time_t)GetTime();
    // Every certificate in the message must be inside its validity window (the reference
    // checks this before the chain walk, paymentrequestplus.cpp:90-101).
    for (const auto& c : certs)
        if (X509_cmp_time(X509_get0_notBefore(c.get()), &now) > 0 || X509_cmp_time(X509_get0_notAfter(c.get()), &now) < 0)
            return fail("certificate expired or not yet active");

    std::unique_ptr<X509_STORE, StoreDeleter> store{X509_STORE_new()};
    if (!store) return fail("error creating X509_STORE");
    for (const auto& d : cs.roots_der)
        if (std::unique_ptr<X509, X509Deleter> x{DecodeDer(d)}) X509_STORE_add_cert(store.get(), x.get());
    if (cs.use_system) X509_STORE_set_default_paths(store.get());

    // the first certificate signs; the rest are untrusted intermediates toward a root
    STACK_OF(X509)* chain = sk_X509_new_null();
    for (size_t i = certs.size() - 1; i > 0; i--) sk_X509_push(chain, certs[i].get());
    std::unique_ptr<X509_STORE_CTX, CtxDeleter> ctx{X509_STORE_CTX_new()};
    bool ok = false;
    std::string e;
    if (!ctx || !X509_STORE_CTX_init(ctx.get(), store.get(), certs[0].get(), chain)) {
        e = "error creating X509_STORE_CTX";
    } else {
        X509_STORE_CTX_set_time(ctx.get(), 0, now);
        const int res = X509_verify_cert(ctx.get());
        const int verr = X509_STORE_CTX_get_error(ctx.get());
        if (res != 1 && !(verr == X509_V_ERR_DEPTH_ZERO_SELF_SIGNED_CERT && cs.allow_self_signed_root)) {
            e = X509_verify_cert_error_string(verr);
        } else {
            // signature over the request with an empty (present) signature field
            PaymentRequest copy = request;
            copy.signature.clear();
            copy.has_signature = true;
            const std::string data = SerializePaymentRequest(copy);
            std::unique_ptr<EVP_PKEY, PkeyDeleter> pub{X509_get_pubkey(certs[0].get())};
            std::unique_ptr<EVP_MD_CTX, MdCtxDeleter> mctx{EVP_MD_CTX_new()};
            if (!pub || !mctx || EVP_DigestVerifyInit(mctx.get(), nullptr, md, nullptr, pub.get()) != 1 ||
                EVP_DigestVerify(mctx.get(), (const unsigned char*)request.signature.data(), request.signature.size(),
                                 (const unsigned char*)data.data(), data.size()) != 1) {
                e = "Bad signature, invalid payment request.";
            } else {
                X509_NAME* name = X509_get_subject_name(certs[0].get());
                const int len = X509_NAME_get_text_by_NID(name, NID_commonName, nullptr, 0);
                if (len > 0) {
                    std::string cn((size_t)len + 1, '\0');
                    if (X509_NAME_get_text_by_NID(name, NID_commonName, &cn[0], len + 1) == len) {
                        cn.resize((size_t)len);
                        merchant = cn;
                        ok = true;
                    }
                }
                if (!ok) e = "Bad certificate, missing common name.";
            }
        }
    }
    sk_X509_free(chain);
    if (!ok) return fail("SSL error: " + e);
    return true;
}

std::vector<std::pair<CScript, Amount>> PaymentRequestPlus::getPayTo() const {
    std::vector<std::pair<CScript, Amount>> out;
    for (const auto& o : details.outputs) {
        const unsigned char* s = (const unsigned char*)o.script.data();
        out.emplace_back(CScript(s, s + o.script.size()), (Amount)o.amount);
    }
    return out;
}

bool VerifyNetwork(const PaymentDetails& d, const std::string& networkId) { return d.network == networkId; }

bool VerifyExpired(const PaymentDetails& d, int64_t now) { return d.has_expires && (int64_t)d.expires < now; }

bool VerifySize(int64_t size) { return size <= BIP70_MAX_PAYMENTREQUEST_SIZE; }

bool VerifyAmount(Amount a) { return MoneyRange(a); }

} // namespace payments
} // namespace bcp
