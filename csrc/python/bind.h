#pragma once
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <string>
#include <vector>

namespace bcp {
namespace py {
namespace pyb = pybind11;

inline std::vector<unsigned char> to_vec(const pyb::bytes& b) {
    std::string s = b;
    return std::vector<unsigned char>(s.begin(), s.end());
}
inline pyb::bytes to_bytes(const unsigned char* p, size_t n) { return pyb::bytes((const char*)p, n); }
inline pyb::bytes to_bytes(const std::vector<unsigned char>& v) { return pyb::bytes((const char*)v.data(), v.size()); }
template <class A> inline pyb::bytes to_bytes(const std::vector<unsigned char, A>& v) {
    return pyb::bytes((const char*)v.data(), v.size());
}

void bind_crypto(pyb::module_& m);
void bind_equihash(pyb::module_& m);
void bind_gpu(pyb::module_& m);
void bind_consensus(pyb::module_& m);
void bind_script(pyb::module_& m);
void bind_node(pyb::module_& m);
void bind_payments(pyb::module_& m);

} // namespace py
} // namespace bcp
