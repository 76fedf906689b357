// Minimal polymorphic message/tag payload standing in for the reference's flatbuffers PMT
// library (pmt/include/pmt/pmtf.hpp:14-104), which is out of scope:
// tags and messages stay host-side control data and never reach a kernel.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <variant>
#include <vector>

namespace pmtf {
class pmt_base
{
public:
    using value_t = std::variant<std::monostate, bool, int64_t, double, std::string, std::vector<float>>;
    pmt_base() = default;
    explicit pmt_base(value_t v) : _v(std::move(v)) {}
    virtual ~pmt_base() = default;
    const value_t& value() const { return _v; }
    bool operator==(const pmt_base& o) const { return _v == o._v; }

private:
    value_t _v;
};
using pmt_sptr = std::shared_ptr<pmt_base>;

template <class T>
inline pmt_sptr make(T v)
{
    return std::make_shared<pmt_base>(pmt_base::value_t(std::move(v)));
}
inline pmt_sptr make(const char* s) { return make(std::string(s)); }
inline pmt_sptr make(int v) { return make(int64_t(v)); }
} // namespace pmtf
