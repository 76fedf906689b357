// Element sizes / type ids for typed ports (reference runtime/lib/parameter_types.cpp).
#include <gnuradio/parameter_types.hpp>

#include <map>
#include <stdexcept>

namespace gr {

size_t parameter_functions::param_size_info(param_type_t p)
{
    switch (p) {
    case param_type_t::FLOAT: return sizeof(float);
    case param_type_t::DOUBLE: return sizeof(double);
    case param_type_t::CFLOAT: return sizeof(gr_complex);
    case param_type_t::CDOUBLE: return sizeof(gr_complexd);
    case param_type_t::INT8: case param_type_t::UINT8: case param_type_t::BOOL: return 1;
    case param_type_t::INT16: case param_type_t::UINT16: return 2;
    case param_type_t::INT32: case param_type_t::UINT32: case param_type_t::ENUM: return 4;
    case param_type_t::INT64: case param_type_t::UINT64: return 8;
    default: return 0;
    }
}

param_type_t parameter_functions::get_param_type_from_typeinfo(std::type_index t)
{
    static const std::map<std::type_index, param_type_t> m = {
        { typeid(float), param_type_t::FLOAT },        { typeid(double), param_type_t::DOUBLE },
        { typeid(gr_complex), param_type_t::CFLOAT },  { typeid(gr_complexd), param_type_t::CDOUBLE },
        { typeid(int8_t), param_type_t::INT8 },        { typeid(int16_t), param_type_t::INT16 },
        { typeid(int32_t), param_type_t::INT32 },      { typeid(int64_t), param_type_t::INT64 },
        { typeid(uint8_t), param_type_t::UINT8 },      { typeid(uint16_t), param_type_t::UINT16 },
        { typeid(uint32_t), param_type_t::UINT32 },    { typeid(uint64_t), param_type_t::UINT64 },
        { typeid(bool), param_type_t::BOOL },
    };
    auto it = m.find(t);
    if (it == m.end()) throw std::invalid_argument("unsupported port data type");
    return it->second;
}

} // namespace gr
