// Python bindings: consensus data model and node subsystems (filled in as they land).
#include "python/bind.h"

namespace bcp {
namespace py {

void bind_consensus(pyb::module_& m) { (void)m; }
void bind_node(pyb::module_& m) { (void)m; }

} // namespace py
} // namespace bcp
