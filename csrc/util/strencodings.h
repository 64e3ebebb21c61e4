// Hex/base32/base64 codecs, money formatting and strict number parsing.
// Behaviour parity: reference src/utilstrencodings.{h,cpp}, src/utilmoneystr.cpp.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace bcp {

bool IsHex(const std::string& str);
bool IsHexNumber(const std::string& str);
std::vector<unsigned char> ParseHex(const std::string& str);
std::string HexStr(const unsigned char* b, const unsigned char* e);
template <typename It, typename = decltype(*std::declval<It>())>
std::string HexStr(It b, It e) {
    if (b == e) return std::string();
    const unsigned char* p = (const unsigned char*)&*b;
    return HexStr(p, p + (e - b));
}
template <typename T> std::string HexStr(const T& v) {
    return HexStr((const unsigned char*)v.data(), (const unsigned char*)v.data() + v.size());
}
std::string EncodeBase64(const unsigned char* p, size_t n);
std::string EncodeBase64(const std::string& s);
std::vector<unsigned char> DecodeBase64(const std::string& s, bool* invalid = nullptr);
std::string EncodeBase32(const unsigned char* p, size_t n);
std::vector<unsigned char> DecodeBase32(const std::string& s, bool* invalid = nullptr);

bool ParseInt32(const std::string& s, int32_t* out);
bool ParseInt64(const std::string& s, int64_t* out);
bool ParseUInt32(const std::string& s, uint32_t* out);
bool ParseDouble(const std::string& s, double* out);
bool ParseFixedPoint(const std::string& val, int decimals, int64_t* amount_out);
int64_t atoi64(const std::string& s);

std::string FormatMoney(int64_t n);
bool ParseMoney(const std::string& s, int64_t& n);

std::string SanitizeString(const std::string& str);
std::string ToLower(std::string s);
std::string ToUpper(std::string s);
std::vector<std::string> SplitString(const std::string& s, char sep);
std::string TrimString(const std::string& s);
std::string strprintf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

} // namespace bcp
