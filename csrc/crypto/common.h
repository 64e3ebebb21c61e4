// Byte-order helpers shared by every hash implementation.
// Behaviour parity: reference src/crypto/common.h (ReadLE32/WriteBE64 etc.).
#pragma once
#include <cstdint>
#include <cstring>

namespace bcp {

static inline uint16_t ReadLE16(const unsigned char* p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t ReadLE32(const unsigned char* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ReadLE64(const unsigned char* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void WriteLE16(unsigned char* p, uint16_t v) { memcpy(p, &v, 2); }
static inline void WriteLE32(unsigned char* p, uint32_t v) { memcpy(p, &v, 4); }
static inline void WriteLE64(unsigned char* p, uint64_t v) { memcpy(p, &v, 8); }
static inline uint32_t ReadBE32(const unsigned char* p) { return __builtin_bswap32(ReadLE32(p)); }
static inline uint64_t ReadBE64(const unsigned char* p) { return __builtin_bswap64(ReadLE64(p)); }
static inline void WriteBE32(unsigned char* p, uint32_t v) { WriteLE32(p, __builtin_bswap32(v)); }
static inline void WriteBE64(unsigned char* p, uint64_t v) { WriteLE64(p, __builtin_bswap64(v)); }

static inline uint32_t Rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline uint32_t Rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static inline uint64_t Rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static inline uint64_t Rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// Zero memory in a way the optimiser cannot elide (reference support/cleanse.cpp).
void memory_cleanse(void* ptr, size_t len);

} // namespace bcp
