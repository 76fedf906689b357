/* Test double of the five RCCL entry points gr::domain_adapter_remote's "rccl" transport calls
 * (newsched_amd/runtime/lib/domain_adapter_remote.cpp, rccl_transport), for 2-process tests of
 * that transport's protocol without two GPUs (tests/test_remote_edge.py; loaded through
 * NSH_RCCL_LIB with NSH_REMOTE_TEST_RCCL=1). Not RCCL: two ranks, one Unix-domain stream socket
 * per communicator (abstract namespace, named by the unique id).
 *
 *   ncclGetUniqueId    a fresh abstract socket name
 *   ncclCommInitRank   rank 0 listens on it and accepts, rank 1 connects (retrying up to 60 s)
 *   ncclSend           host ring (stream NULL): copies the payload when called. Device ring: a
 *                      hipMemcpyAsync D2H into pinned memory on the caller's stream and an event
 *                      behind it -- the payload is read in stream order, as RCCL reads it, so the
 *                      caller may release its span at once. A writer thread sends the payloads in
 *                      call order (waiting for each one's event first).
 *   ncclRecv           receives the payload; device ring: then a hipMemcpyAsync H2D on the
 *                      caller's stream (the landing is ordered before later work on that stream,
 *                      as RCCL's), synchronised before the staging is freed
 *   ncclCommDestroy    lets the writer finish, then closes
 * HIP is loaded with dlopen only when a device ring uses it (the CPU tests run without a GPU).
 * Errors are nonzero returns; ncclGetErrorString names them. A peer that went away makes the
 * writer drop what is left (no SIGPIPE: MSG_NOSIGNAL). */
#include <dlfcn.h>
#include <errno.h>
#include <stddef.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

typedef struct {
    char internal[128];
} ncclUniqueId;

typedef struct job {
    struct job* next;
    size_t n;
    void* ev;     /* device payload: wait for this event before sending */
    char* pinned; /* device payload: the staging (hipHostFree after sending) */
    char data[];
} job;

/* the HIP runtime, for device payloads */
typedef struct {
    int (*memcpy_async)(void*, const void*, size_t, int, void*);
    int (*host_malloc)(void**, size_t, unsigned);
    int (*host_free)(void*);
    int (*event_create)(void**, unsigned);
    int (*event_record)(void*, void*);
    int (*event_sync)(void*);
    int (*event_destroy)(void*);
    int (*stream_sync)(void*);
} hipapi;
static hipapi* hip(void)
{
    static hipapi a;
    static int state = 0; /* 0 untried, 1 ok, -1 unavailable */
    static pthread_mutex_t m = PTHREAD_MUTEX_INITIALIZER;
    pthread_mutex_lock(&m);
    if (state == 0) {
        void* h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
        state = -1;
        if (h) {
            *(void**)&a.memcpy_async = dlsym(h, "hipMemcpyAsync");
            *(void**)&a.host_malloc = dlsym(h, "hipHostMalloc");
            *(void**)&a.host_free = dlsym(h, "hipHostFree");
            *(void**)&a.event_create = dlsym(h, "hipEventCreateWithFlags");
            *(void**)&a.event_record = dlsym(h, "hipEventRecord");
            *(void**)&a.event_sync = dlsym(h, "hipEventSynchronize");
            *(void**)&a.event_destroy = dlsym(h, "hipEventDestroy");
            *(void**)&a.stream_sync = dlsym(h, "hipStreamSynchronize");
            if (a.memcpy_async && a.host_malloc && a.host_free && a.event_create && a.event_record && a.event_sync &&
                a.event_destroy && a.stream_sync)
                state = 1;
        }
    }
    pthread_mutex_unlock(&m);
    return state == 1 ? &a : NULL;
}
enum { H2D = 1, D2H = 2, EVENT_DISABLE_TIMING = 2 };

typedef struct {
    int fd;
    int rank;
    pthread_t writer;
    pthread_mutex_t m;
    pthread_cond_t cv;
    job *head, *tail;
    int stop, broken;
} fcomm;

enum { OK = 0, E_SYS = 2, E_ARG = 4 };

static void sock_name(const ncclUniqueId* id, struct sockaddr_un* a, socklen_t* len)
{
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    const size_t n = strnlen(id->internal, sizeof(a->sun_path) - 2);
    memcpy(a->sun_path + 1, id->internal, n); /* abstract: leading NUL, no file */
    *len = (socklen_t)(offsetof(struct sockaddr_un, sun_path) + 1 + n);
}

static void* writer_main(void* arg)
{
    fcomm* c = (fcomm*)arg;
    for (;;) {
        pthread_mutex_lock(&c->m);
        while (!c->head && !c->stop) pthread_cond_wait(&c->cv, &c->m);
        job* j = c->head;
        if (!j) { /* stop requested and drained */
            pthread_mutex_unlock(&c->m);
            return NULL;
        }
        c->head = j->next;
        if (!c->head) c->tail = NULL;
        pthread_mutex_unlock(&c->m);
        const char* src = j->data;
        if (j->ev) { /* device payload: its stream-ordered D2H copy has to land first */
            if (hip()->event_sync(j->ev) != 0) c->broken = 1;
            hip()->event_destroy(j->ev);
            src = j->pinned;
        }
        size_t off = 0;
        while (off < j->n && !c->broken) {
            const ssize_t w = send(c->fd, src + off, j->n - off, MSG_NOSIGNAL);
            if (w > 0)
                off += (size_t)w;
            else if (w < 0 && errno == EINTR)
                continue;
            else
                c->broken = 1;
        }
        if (j->pinned) hip()->host_free(j->pinned);
        free(j);
    }
}

int ncclGetUniqueId(ncclUniqueId* id)
{
    static int counter = 0;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    memset(id, 0, sizeof(*id));
    snprintf(id->internal, sizeof(id->internal), "nsh_fake_rccl_%d_%ld_%ld_%d", (int)getpid(), (long)ts.tv_sec,
             (long)ts.tv_nsec, __atomic_fetch_add(&counter, 1, __ATOMIC_RELAXED));
    return OK;
}

int ncclCommInitRank(void** comm, int nranks, ncclUniqueId id, int rank)
{
    if (!comm || nranks != 2 || rank < 0 || rank > 1) return E_ARG;
    struct sockaddr_un a;
    socklen_t len;
    sock_name(&id, &a, &len);
    int fd = -1;
    if (rank == 0) {
        const int l = socket(AF_UNIX, SOCK_STREAM, 0);
        if (l < 0) return E_SYS;
        if (bind(l, (struct sockaddr*)&a, len) != 0 || listen(l, 1) != 0) {
            close(l);
            return E_SYS;
        }
        fd = accept(l, NULL, NULL);
        close(l);
    } else {
        for (int tries = 0; tries < 6000; ++tries) { /* 60 s */
            fd = socket(AF_UNIX, SOCK_STREAM, 0);
            if (fd < 0) return E_SYS;
            if (connect(fd, (struct sockaddr*)&a, len) == 0) break;
            close(fd);
            fd = -1;
            usleep(10000);
        }
    }
    if (fd < 0) return E_SYS;
    fcomm* c = (fcomm*)calloc(1, sizeof(fcomm));
    c->fd = fd;
    c->rank = rank;
    pthread_mutex_init(&c->m, NULL);
    pthread_cond_init(&c->cv, NULL);
    pthread_create(&c->writer, NULL, writer_main, c);
    *comm = c;
    return OK;
}

int ncclSend(const void* buf, size_t count, int datatype, int peer, void* comm, void* stream)
{
    fcomm* c = (fcomm*)comm;
    if (!c || datatype != 0 || peer != 1 - c->rank || (!buf && count)) return E_ARG;
    if (c->broken) return E_SYS;
    job* j = (job*)calloc(1, sizeof(job) + (stream ? 0 : count));
    if (!j) return E_SYS;
    j->n = count;
    if (!stream) {
        memcpy(j->data, buf, count);
    } else {
        hipapi* h = hip();
        if (!h || h->host_malloc((void**)&j->pinned, count ? count : 1, 0) != 0) {
            free(j);
            return E_SYS;
        }
        if (h->memcpy_async(j->pinned, buf, count, D2H, stream) != 0 || h->event_create(&j->ev, EVENT_DISABLE_TIMING) != 0 ||
            h->event_record(j->ev, stream) != 0) {
            if (j->ev) h->event_destroy(j->ev);
            h->host_free(j->pinned);
            free(j);
            return E_SYS;
        }
    }
    pthread_mutex_lock(&c->m);
    if (c->tail)
        c->tail->next = j;
    else
        c->head = j;
    c->tail = j;
    pthread_cond_signal(&c->cv);
    pthread_mutex_unlock(&c->m);
    return OK;
}

int ncclRecv(void* buf, size_t count, int datatype, int peer, void* comm, void* stream)
{
    fcomm* c = (fcomm*)comm;
    if (!c || datatype != 0 || peer != 1 - c->rank || (!buf && count)) return E_ARG;
    hipapi* h = stream ? hip() : NULL;
    char* dst = (char*)buf;
    if (stream && (!h || h->host_malloc((void**)&dst, count ? count : 1, 0) != 0)) return E_SYS;
    size_t off = 0;
    int rc = OK;
    while (off < count) {
        const ssize_t r = recv(c->fd, dst + off, count - off, 0);
        if (r > 0)
            off += (size_t)r;
        else if (r < 0 && errno == EINTR)
            continue;
        else {
            rc = E_SYS;
            break;
        }
    }
    if (stream) {
        if (rc == OK && (h->memcpy_async(buf, dst, count, H2D, stream) != 0 || h->stream_sync(stream) != 0)) rc = E_SYS;
        h->host_free(dst);
    }
    return rc;
}

int ncclCommDestroy(void* comm)
{
    fcomm* c = (fcomm*)comm;
    if (!c) return OK;
    pthread_mutex_lock(&c->m);
    c->stop = 1;
    pthread_cond_signal(&c->cv);
    pthread_mutex_unlock(&c->m);
    pthread_join(c->writer, NULL);
    close(c->fd);
    pthread_mutex_destroy(&c->m);
    pthread_cond_destroy(&c->cv);
    free(c);
    return OK;
}

const char* ncclGetErrorString(int r)
{
    return r == E_ARG ? "fake rccl: invalid argument" : r == E_SYS ? "fake rccl: system error (peer gone?)" : "fake rccl: ok";
}
