// Port/parameter element types (reference runtime/include/gnuradio/parameter_types.hpp,
// runtime/lib/parameter_types.cpp): a port's item size is sizeof(T) times the product of
// its dims (reference port.hpp:57-64).
#pragma once
#include <cstddef>
#include <gnuradio/types.hpp>
#include <typeindex>

namespace gr {

enum class param_type_t {
    UNTYPED, FLOAT, DOUBLE, CFLOAT, CDOUBLE, INT8, INT16, INT32, INT64,
    UINT8, UINT16, UINT32, UINT64, BOOL, ENUM, STRING, VOID
};

struct parameter_functions {
    static size_t param_size_info(param_type_t p);
    static param_type_t get_param_type_from_typeinfo(std::type_index t);
};

} // namespace gr
