// Native planner of MemorySystem.consolidate_batch (batch_plan.cpp).
#pragma once
#include <pybind11/pybind11.h>

namespace lzrt {
void register_batch_plan(pybind11::module_& m);
}
