// Wallet encryption.
// Parity: reference src/wallet/crypter.{h,cpp}: CMasterKey (encrypted master key,
// salt, derivation method 0 = EVP_sha512-style iterated SHA-512, iteration count),
// CCrypter::SetKeyFromPassphrase (BytesToKeySHA512AES), AES-256-CBC encrypt/decrypt
// of secrets with IV = first 16 bytes of the pubkey's SHA256d, and CCryptoKeyStore
// (lock/unlock, encrypted key map, plain keys before encryption).
#pragma once
#include "keys/key.h"
#include "script/sign.h"
#include "util/lockedpool.h"

#include <map>
#include <string>
#include <vector>

namespace bcp {

static const unsigned int WALLET_CRYPTO_KEY_SIZE = 32;
static const unsigned int WALLET_CRYPTO_SALT_SIZE = 8;
static const unsigned int WALLET_CRYPTO_IV_SIZE = 16;

typedef std::vector<unsigned char, secure_allocator<unsigned char>> CKeyingMaterial; // mlocked, cleansed on free

class CMasterKey {
public:
    std::vector<unsigned char> vchCryptedKey;
    std::vector<unsigned char> vchSalt;
    unsigned int nDerivationMethod = 0; // 0 = iterated SHA-512
    unsigned int nDeriveIterations = 25000;
    std::vector<unsigned char> vchOtherDerivationParameters;

    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, vchCryptedKey);
        ::bcp::Serialize(s, vchSalt);
        ::bcp::Serialize(s, nDerivationMethod);
        ::bcp::Serialize(s, nDeriveIterations);
        ::bcp::Serialize(s, vchOtherDerivationParameters);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, vchCryptedKey);
        ::bcp::Unserialize(s, vchSalt);
        ::bcp::Unserialize(s, nDerivationMethod);
        ::bcp::Unserialize(s, nDeriveIterations);
        ::bcp::Unserialize(s, vchOtherDerivationParameters);
    }
};

class CCrypter {
public:
    CCrypter() { Clear(); }
    ~CCrypter() { Clear(); }
    bool SetKeyFromPassphrase(const std::string& passphrase, const std::vector<unsigned char>& salt,
                              unsigned int rounds, unsigned int method);
    bool SetKey(const CKeyingMaterial& key, const std::vector<unsigned char>& iv);
    bool Encrypt(const CKeyingMaterial& plain, std::vector<unsigned char>& cipher) const;
    bool Decrypt(const std::vector<unsigned char>& cipher, CKeyingMaterial& plain) const;
    void Clear();

private:
    friend struct CrypterTestAccess; // wallet_crypto tests compare the derived key and IV with OpenSSL
    unsigned char vchKey[WALLET_CRYPTO_KEY_SIZE];
    unsigned char vchIV[WALLET_CRYPTO_IV_SIZE];
    bool fKeySet = false;
};

bool EncryptSecret(const CKeyingMaterial& masterKey, const CKeyingMaterial& plain, const uint256& iv,
                   std::vector<unsigned char>& cipher);
bool DecryptSecret(const CKeyingMaterial& masterKey, const std::vector<unsigned char>& cipher, const uint256& iv,
                   CKeyingMaterial& plain);

// Key store that keeps private keys encrypted under a master key once encrypted.
class CCryptoKeyStore : public CBasicKeyStore {
public:
    bool IsCrypted() const { return fUseCrypto; }
    bool IsLocked() const;
    bool Lock();
    bool AddKeyPubKey(const CKey& key, const CPubKey& pubkey) override;
    virtual bool AddCryptedKey(const CPubKey& pubkey, const std::vector<unsigned char>& crypted);
    bool HaveKey(const CKeyID& address) const override;
    bool GetKey(const CKeyID& address, CKey& keyOut) const override;
    bool GetPubKey(const CKeyID& address, CPubKey& out) const override;
    std::set<CKeyID> GetKeys() const override;
    const std::map<CKeyID, std::pair<CPubKey, std::vector<unsigned char>>>& CryptedKeys() const { return mapCryptedKeys; }

protected:
    bool SetCrypted();
    bool EncryptKeys(const CKeyingMaterial& masterKeyIn); // move plain keys into the crypted map
    bool Unlock(const CKeyingMaterial& masterKeyIn);
    CKeyingMaterial vMasterKey;
    std::map<CKeyID, std::pair<CPubKey, std::vector<unsigned char>>> mapCryptedKeys;

private:
    bool fUseCrypto = false;
    bool fDecryptionThoroughlyChecked = false;
};

} // namespace bcp
