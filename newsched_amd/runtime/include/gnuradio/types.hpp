// Stream element types (reference runtime/include/gnuradio/types.hpp:15).
#pragma once
#include <complex>
#include <cstddef>
#include <cstdint>
#include <vector>

typedef std::complex<float> gr_complex;   // interleaved (re, im) fp32, 8 B per sample
typedef std::complex<double> gr_complexd;
typedef std::vector<int> gr_vector_int;
typedef std::vector<unsigned int> gr_vector_uint;
typedef std::vector<float> gr_vector_float;
typedef std::vector<double> gr_vector_double;
typedef std::vector<void*> gr_vector_void_star;
typedef std::vector<const void*> gr_vector_const_void_star;
