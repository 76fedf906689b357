// Per-block attribute dictionary (reference runtime/include/gnuradio/gpdict.hpp).
#pragma once
#include <map>
#include <mutex>
#include <string>

namespace gr {
class gpdict
{
public:
    void set_int_value(const std::string& k, int v)
    {
        std::lock_guard<std::mutex> g(_m);
        _ints[k] = v;
    }
    int get_int_value(const std::string& k)
    {
        std::lock_guard<std::mutex> g(_m);
        auto it = _ints.find(k);
        return it == _ints.end() ? 0 : it->second;
    }

private:
    std::mutex _m;
    std::map<std::string, int> _ints;
};
} // namespace gr
