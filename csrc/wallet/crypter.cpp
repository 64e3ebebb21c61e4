#include "wallet/crypter.h"
#include "crypto/hashes.h"
#include "util/util.h"

#include <cstring>

namespace bcp {

// EVP_BytesToKey-compatible derivation with SHA-512 (reference crypter.cpp:18-44).
static int BytesToKeySHA512AES(const std::vector<unsigned char>& salt, const std::string& data, int count,
                               unsigned char* key, unsigned char* iv) {
    if (!count || !key || !iv) return 0;
    unsigned char buf[CSHA512::OUTPUT_SIZE];
    CSHA512 di;
    di.Write((const unsigned char*)data.data(), data.size());
    if (!salt.empty()) di.Write(salt.data(), salt.size());
    di.Finalize(buf);
    for (int i = 0; i != count - 1; i++) di.Reset().Write(buf, sizeof(buf)).Finalize(buf);
    memcpy(key, buf, WALLET_CRYPTO_KEY_SIZE);
    memcpy(iv, buf + WALLET_CRYPTO_KEY_SIZE, WALLET_CRYPTO_IV_SIZE);
    memset(buf, 0, sizeof(buf));
    return WALLET_CRYPTO_KEY_SIZE;
}

void CCrypter::Clear() {
    memset(vchKey, 0, sizeof(vchKey));
    memset(vchIV, 0, sizeof(vchIV));
    fKeySet = false;
}

bool CCrypter::SetKeyFromPassphrase(const std::string& passphrase, const std::vector<unsigned char>& salt,
                                    unsigned int rounds, unsigned int method) {
    if (rounds < 1 || salt.size() != WALLET_CRYPTO_SALT_SIZE) return false;
    int i = 0;
    if (method == 0) i = BytesToKeySHA512AES(salt, passphrase, (int)rounds, vchKey, vchIV);
    if (i != (int)WALLET_CRYPTO_KEY_SIZE) {
        Clear();
        return false;
    }
    fKeySet = true;
    return true;
}

bool CCrypter::SetKey(const CKeyingMaterial& key, const std::vector<unsigned char>& iv) {
    if (key.size() != WALLET_CRYPTO_KEY_SIZE || iv.size() != WALLET_CRYPTO_IV_SIZE) return false;
    memcpy(vchKey, key.data(), key.size());
    memcpy(vchIV, iv.data(), iv.size());
    fKeySet = true;
    return true;
}

bool CCrypter::Encrypt(const CKeyingMaterial& plain, std::vector<unsigned char>& cipher) const {
    if (!fKeySet) return false;
    cipher.resize(plain.size() + 16); // max PKCS7 padding
    AES256CBCEncrypt enc(vchKey, vchIV, true);
    const int n = enc.Encrypt(plain.data(), (int)plain.size(), cipher.data());
    if (n < (int)plain.size()) return false;
    cipher.resize(n);
    return true;
}

bool CCrypter::Decrypt(const std::vector<unsigned char>& cipher, CKeyingMaterial& plain) const {
    if (!fKeySet) return false;
    plain.resize(cipher.size());
    AES256CBCDecrypt dec(vchKey, vchIV, true);
    const int n = dec.Decrypt(cipher.data(), (int)cipher.size(), plain.data());
    if (n == 0) return false;
    plain.resize(n);
    return true;
}

bool EncryptSecret(const CKeyingMaterial& masterKey, const CKeyingMaterial& plain, const uint256& iv,
                   std::vector<unsigned char>& cipher) {
    CCrypter c;
    std::vector<unsigned char> vIV(iv.begin(), iv.begin() + WALLET_CRYPTO_IV_SIZE);
    if (!c.SetKey(masterKey, vIV)) return false;
    return c.Encrypt(plain, cipher);
}

bool DecryptSecret(const CKeyingMaterial& masterKey, const std::vector<unsigned char>& cipher, const uint256& iv,
                   CKeyingMaterial& plain) {
    CCrypter c;
    std::vector<unsigned char> vIV(iv.begin(), iv.begin() + WALLET_CRYPTO_IV_SIZE);
    if (!c.SetKey(masterKey, vIV)) return false;
    return c.Decrypt(cipher, plain);
}

static bool DecryptKey(const CKeyingMaterial& masterKey, const std::vector<unsigned char>& crypted,
                       const CPubKey& pub, CKey& key) {
    CKeyingMaterial secret;
    if (!DecryptSecret(masterKey, crypted, pub.GetHash(), secret)) return false;
    if (secret.size() != 32) return false;
    key.Set(secret.begin(), secret.end(), pub.IsCompressed());
    return key.VerifyPubKey(pub);
}

bool CCryptoKeyStore::SetCrypted() {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (fUseCrypto) return true;
    if (!mapKeys.empty()) return false;
    fUseCrypto = true;
    return true;
}

bool CCryptoKeyStore::IsLocked() const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    return fUseCrypto && vMasterKey.empty();
}

bool CCryptoKeyStore::Lock() {
    if (!SetCrypted()) return false;
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    std::fill(vMasterKey.begin(), vMasterKey.end(), 0);
    vMasterKey.clear();
    return true;
}

bool CCryptoKeyStore::Unlock(const CKeyingMaterial& masterKeyIn) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!SetCrypted()) return false;
    bool keyPass = false, keyFail = false;
    for (const auto& kv : mapCryptedKeys) {
        CKey key;
        if (!DecryptKey(masterKeyIn, kv.second.second, kv.second.first, key)) {
            keyFail = true;
            break;
        }
        keyPass = true;
        if (fDecryptionThoroughlyChecked) break;
    }
    if (keyPass && keyFail) {
        LogPrintf("The wallet is probably corrupted: Some keys decrypt but not all.\n");
        return false;
    }
    if (keyFail || (!keyPass && !mapCryptedKeys.empty())) return false;
    vMasterKey = masterKeyIn;
    fDecryptionThoroughlyChecked = true;
    return true;
}

bool CCryptoKeyStore::AddKeyPubKey(const CKey& key, const CPubKey& pubkey) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!IsCrypted()) return CBasicKeyStore::AddKeyPubKey(key, pubkey);
    if (IsLocked()) return false;
    std::vector<unsigned char> crypted;
    CKeyingMaterial secret(key.begin(), key.begin() + 32);
    if (!EncryptSecret(vMasterKey, secret, pubkey.GetHash(), crypted)) return false;
    return AddCryptedKey(pubkey, crypted);
}

bool CCryptoKeyStore::AddCryptedKey(const CPubKey& pubkey, const std::vector<unsigned char>& crypted) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!SetCrypted()) return false;
    mapCryptedKeys[pubkey.GetID()] = {pubkey, crypted};
    return true;
}

bool CCryptoKeyStore::HaveKey(const CKeyID& address) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!IsCrypted()) return CBasicKeyStore::HaveKey(address);
    return mapCryptedKeys.count(address) > 0;
}

bool CCryptoKeyStore::GetKey(const CKeyID& address, CKey& keyOut) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!IsCrypted()) return CBasicKeyStore::GetKey(address, keyOut);
    auto it = mapCryptedKeys.find(address);
    if (it == mapCryptedKeys.end() || vMasterKey.empty()) return false;
    return DecryptKey(vMasterKey, it->second.second, it->second.first, keyOut);
}

bool CCryptoKeyStore::GetPubKey(const CKeyID& address, CPubKey& out) const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!IsCrypted()) return CBasicKeyStore::GetPubKey(address, out);
    auto it = mapCryptedKeys.find(address);
    if (it != mapCryptedKeys.end()) {
        out = it->second.first;
        return true;
    }
    // watch-only pubkeys
    return CBasicKeyStore::GetPubKey(address, out);
}

std::set<CKeyID> CCryptoKeyStore::GetKeys() const {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!IsCrypted()) return CBasicKeyStore::GetKeys();
    std::set<CKeyID> s;
    for (const auto& kv : mapCryptedKeys) s.insert(kv.first);
    return s;
}

bool CCryptoKeyStore::EncryptKeys(const CKeyingMaterial& masterKeyIn) {
    std::lock_guard<CCriticalSection> l(cs_KeyStore);
    if (!mapCryptedKeys.empty() || IsCrypted()) return false;
    fUseCrypto = true;
    for (const auto& kv : mapKeys) {
        const CKey& key = kv.second;
        const CPubKey pub = key.GetPubKey();
        CKeyingMaterial secret(key.begin(), key.begin() + 32);
        std::vector<unsigned char> crypted;
        if (!EncryptSecret(masterKeyIn, secret, pub.GetHash(), crypted)) return false;
        if (!AddCryptedKey(pub, crypted)) return false;
    }
    mapKeys.clear();
    return true;
}

} // namespace bcp
