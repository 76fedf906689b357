// Host double-mapped circular buffer: the scheduler_mt default edge buffer and the CPU
// baseline's (reference runtime/include/gnuradio/vmcircbuf.hpp, runtime/lib/vmcircbuf.cpp,
// vmcircbuf_sysv_shm.cpp, vmcircbuf_mmap_shm_open.cpp). One memfd mapped twice back to
// back, so every read/write span is contiguous. Readable = written - read; writable =
// min(capacity - size - 1, capacity / 2) (reference vmcircbuf.cpp:79-83). The byte size
// is rounded up to a whole number of pages.
#pragma once
#include <gnuradio/buffer.hpp>

namespace gr {

enum class vmcirc_buffer_type { AUTO, SYSV_SHM, MMAP_SHM, MMAP_TMPFILE };

class vmcirc_buffer_properties : public buffer_properties
{
public:
    explicit vmcirc_buffer_properties(vmcirc_buffer_type t = vmcirc_buffer_type::AUTO) : _t(t) {}
    vmcirc_buffer_type buffer_type() const { return _t; }
    static std::shared_ptr<buffer_properties> make(vmcirc_buffer_type t)
    {
        return std::make_shared<vmcirc_buffer_properties>(t);
    }

private:
    vmcirc_buffer_type _t;
};

class vmcirc_buffer : public buffer
{
public:
    using sptr = std::shared_ptr<vmcirc_buffer>;
    static buffer_sptr make(size_t num_items, size_t item_size, std::shared_ptr<buffer_properties> props);
    vmcirc_buffer(size_t num_items, size_t item_size);
    ~vmcirc_buffer() override;

    int size();      // items readable
    int capacity();  // items
    void* read_ptr() override;
    void* write_ptr() override;
    bool read_info(buffer_info_t& info) override;
    bool write_info(buffer_info_t& info) override;
    void post_read(int num_items) override;
    void post_write(int num_items) override;
    void copy_items(std::shared_ptr<buffer> from, int nitems) override;
    void discard_unread() override;

protected:
    uint8_t* _buffer = nullptr; // 2 * _buf_size bytes of address space
    size_t _num_items;
    size_t _item_size;
    size_t _buf_size;
};

} // namespace gr

#define VMCIRC_BUFFER_ARGS gr::vmcirc_buffer::make, gr::vmcirc_buffer_properties::make(gr::vmcirc_buffer_type::AUTO)
#define VMCIRC_BUFFER_SYSV_SHM_ARGS \
    gr::vmcirc_buffer::make, gr::vmcirc_buffer_properties::make(gr::vmcirc_buffer_type::SYSV_SHM)
#define VMCIRC_BUFFER_MMAP_SHM_ARGS \
    gr::vmcirc_buffer::make, gr::vmcirc_buffer_properties::make(gr::vmcirc_buffer_type::MMAP_SHM)
