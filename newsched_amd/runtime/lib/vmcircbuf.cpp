// Host double-mapped ring (reference runtime/lib/vmcircbuf.cpp:16-125 and the SysV /
// shm_open mappers vmcircbuf_sysv_shm.cpp:22-155, vmcircbuf_mmap_shm_open.cpp:21-155),
// restated with memfd_create: reserve 2x the size, map the same file into both halves.
#include <gnuradio/vmcircbuf.hpp>

#include <cstring>
#include <numeric>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace gr {

namespace {
size_t page_size()
{
    static const size_t p = (size_t)sysconf(_SC_PAGESIZE);
    return p;
}
} // namespace

buffer_sptr vmcirc_buffer::make(size_t num_items, size_t item_size, std::shared_ptr<buffer_properties> props)
{
    if (props && !std::dynamic_pointer_cast<vmcirc_buffer_properties>(props))
        throw std::runtime_error("Failed to cast buffer properties to vmcirc_buffer_properties");
    return std::make_shared<vmcirc_buffer>(num_items, item_size);
}

vmcirc_buffer::vmcirc_buffer(size_t num_items, size_t item_size) : _item_size(item_size)
{
    if (item_size == 0) throw std::invalid_argument("vmcirc_buffer: item_size 0");
    // smallest item count >= num_items whose byte size is a whole number of pages
    const size_t unit = std::lcm(page_size(), item_size) / item_size;
    _num_items = (std::max<size_t>(num_items, 1) + unit - 1) / unit * unit;
    _buf_size = _num_items * item_size;

    const int fd = (int)syscall(SYS_memfd_create, "newsched_vmcirc", 0);
    if (fd < 0) throw std::runtime_error("vmcirc_buffer: memfd_create failed");
    if (ftruncate(fd, (off_t)_buf_size) != 0) {
        close(fd);
        throw std::runtime_error("vmcirc_buffer: ftruncate failed");
    }
    void* base = mmap(nullptr, 2 * _buf_size, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (base == MAP_FAILED) {
        close(fd);
        throw std::runtime_error("vmcirc_buffer: address reservation failed");
    }
    void* a = mmap(base, _buf_size, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0);
    void* b = mmap((uint8_t*)base + _buf_size, _buf_size, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0);
    close(fd);
    if (a == MAP_FAILED || b == MAP_FAILED) {
        munmap(base, 2 * _buf_size);
        throw std::runtime_error("vmcirc_buffer: double mapping failed");
    }
    _buffer = (uint8_t*)base;
    set_type("vmcirc_buffer");
}

vmcirc_buffer::~vmcirc_buffer()
{
    if (_buffer) munmap(_buffer, 2 * _buf_size);
}

int vmcirc_buffer::size() { return (int)(_total_written - _total_read); }
int vmcirc_buffer::capacity() { return (int)_num_items; }
void* vmcirc_buffer::read_ptr() { return _buffer + (_total_read % _num_items) * _item_size; }
void* vmcirc_buffer::write_ptr() { return _buffer + (_total_written % _num_items) * _item_size; }

bool vmcirc_buffer::read_info(buffer_info_t& info)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    info.ptr = read_ptr();
    info.n_items = size();
    info.item_size = _item_size;
    info.total_items = (int)_total_read;
    return true;
}

bool vmcirc_buffer::write_info(buffer_info_t& info)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    info.ptr = write_ptr();
    int n = capacity() - size() - 1;          // keep one slot between writer and reader
    n = std::min(n, capacity() / 2);          // half-full cap (reference vmcircbuf.cpp:83)
    info.n_items = std::max(n, 0);
    info.item_size = _item_size;
    info.total_items = (int)_total_written;
    return true;
}

void vmcirc_buffer::discard_unread()
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    drop_unread_locked();
}

void vmcirc_buffer::post_read(int n)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    _total_read += (uint64_t)n;
}

void vmcirc_buffer::post_write(int n)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    _total_written += (uint64_t)n;
}

void vmcirc_buffer::copy_items(std::shared_ptr<buffer> from, int nitems)
{
    std::lock_guard<std::mutex> g(_buf_mutex);
    std::memcpy(write_ptr(), from->write_ptr(), (size_t)nitems * _item_size);
}

} // namespace gr
