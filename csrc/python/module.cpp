// pybind11 entry point for bitcoincashplus_amd._bcpnative.
// Each subsystem registers its own bindings (bind_*.cpp) so the module stays modular.
#include "python/bind.h"

PYBIND11_MODULE(_bcpnative, m) {
    m.doc() = "bitcoincashplus_amd native core: consensus C++ + CDNA4 HIP kernels";
    bcp::py::bind_crypto(m);
    bcp::py::bind_equihash(m);
    bcp::py::bind_gpu(m);
    bcp::py::bind_consensus(m);
    bcp::py::bind_script(m);
    bcp::py::bind_node(m);
    bcp::py::bind_payments(m);
}
