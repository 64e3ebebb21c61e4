// Python bindings: node subsystems (filled in as they land).
#include "python/bind.h"

namespace bcp {
namespace py {

void bind_node(pyb::module_& m) { (void)m; }

} // namespace py
} // namespace bcp
