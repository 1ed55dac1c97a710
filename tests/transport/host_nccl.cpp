// host_nccl.cpp -- test transport: the subset of the NCCL/RCCL API that comm.cpp resolves (ncclGetUniqueId,
// ncclCommInitRank, ncclCommDestroy, ncclAllGather, ncclSend, ncclRecv, ncclGroupStart/End,
// ncclGetErrorString), carried over Unix-domain sockets through host memory.
//
// RCCL refuses two ranks on one device ("Duplicate GPU detected"), so on a one-GPU box the multi-rank RCCL
// path of comm.cpp (the all-gather slot layout, the grouped halo send/recv pairing, the rank-order folds) can
// only run with another transport underneath. libcwf_hip.so loads this library instead of librccl when
// CWF_RCCL_LIB names it (knobs.hpp); tests/test_gpu_transport.py runs 2 and 3 processes on one GPU through it.
// Semantics kept: a group's operations run at ncclGroupEnd; sends and receives between a pair of ranks
// match in issue order; an all-gather places rank r's chunk at recvbuff + r * count. Not a product path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace
{
struct HostComm
{
    int n = 0, rank = 0, listen_fd = -1;
    std::string dir;
    std::vector<int> fd;  // socket to each peer (-1 for self)
};

struct Op
{
    enum Kind
    {
        kAllGather,
        kSend,
        kRecv
    } kind;
    const void *src;
    void *dst;
    size_t bytes;  // per rank for an all-gather
    int peer;
    HostComm *comm;
    hipStream_t stream;
};

thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

size_t type_bytes(ncclDataType_t t)
{
    switch (t)
    {
    case ncclInt8:
    case ncclUint8:
        return 1;
    case ncclFloat16:
    case ncclBfloat16:
        return 2;
    case ncclInt32:
    case ncclUint32:
    case ncclFloat32:
        return 4;
    case ncclInt64:
    case ncclUint64:
    case ncclFloat64:
        return 8;
    default:
        return 0;
    }
}

bool write_all(int fd, const void *p, size_t n)
{
    const char *c = static_cast<const char *>(p);
    while (n)
    {
        const ssize_t w = ::write(fd, c, n);
        if (w <= 0)
            return false;
        c += w;
        n -= (size_t)w;
    }
    return true;
}

bool read_all(int fd, void *p, size_t n)
{
    char *c = static_cast<char *>(p);
    while (n)
    {
        const ssize_t r = ::read(fd, c, n);
        if (r <= 0)
            return false;
        c += r;
        n -= (size_t)r;
    }
    return true;
}

sockaddr_un addr_of(const std::string &dir, int rank)
{
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    snprintf(a.sun_path, sizeof a.sun_path, "%s/r%d", dir.c_str(), rank);
    return a;
}

// Every op's staged bytes, exchanged pairwise in ascending peer order (the lower rank of a pair writes first),
// which cannot deadlock: all ranks walk their peers in the same total order.
ncclResult_t run(std::vector<Op> &ops)
{
    if (ops.empty())
        return ncclSuccess;
    HostComm *c = ops[0].comm;
    for (const Op &o : ops)
        if (o.comm != c)
            return ncclInvalidUsage;  // one communicator per group (all comm.cpp issues)
    for (const Op &o : ops)
        if (hipStreamSynchronize(o.stream) != hipSuccess)
            return ncclUnhandledCudaError;
    std::vector<std::vector<char>> out(c->n);  // bytes to each peer, op order
    std::vector<size_t> in_bytes(c->n, 0);
    for (const Op &o : ops)
    {
        if (o.kind == Op::kRecv)
        {
            in_bytes[o.peer] += o.bytes;
            continue;
        }
        std::vector<char> h(o.bytes);
        if (o.bytes && hipMemcpy(h.data(), o.src, o.bytes, hipMemcpyDeviceToHost) != hipSuccess)
            return ncclUnhandledCudaError;
        if (o.kind == Op::kSend)
            out[o.peer].insert(out[o.peer].end(), h.begin(), h.end());
        else
        {
            for (int p = 0; p < c->n; ++p)
                if (p != c->rank)
                {
                    out[p].insert(out[p].end(), h.begin(), h.end());
                    in_bytes[p] += o.bytes;
                }
            char *own = static_cast<char *>(o.dst) + (size_t)c->rank * o.bytes;
            if (own != o.src && o.bytes && hipMemcpy(own, o.src, o.bytes, hipMemcpyDeviceToDevice) != hipSuccess)
                return ncclUnhandledCudaError;
        }
    }
    std::vector<std::vector<char>> in(c->n);
    for (int p = 0; p < c->n; ++p)
    {
        if (p == c->rank)
            continue;
        in[p].resize(in_bytes[p]);
        const bool first_write = c->rank < p;
        if (first_write && !write_all(c->fd[p], out[p].data(), out[p].size()))
            return ncclSystemError;
        if (!read_all(c->fd[p], in[p].data(), in[p].size()))
            return ncclSystemError;
        if (!first_write && !write_all(c->fd[p], out[p].data(), out[p].size()))
            return ncclSystemError;
    }
    std::vector<size_t> at(c->n, 0);
    for (const Op &o : ops)
    {
        if (o.kind == Op::kSend)
            continue;
        for (int p = 0; p < c->n; ++p)
        {
            if (p == c->rank || (o.kind == Op::kRecv && p != o.peer))
                continue;
            char *dst = static_cast<char *>(o.dst) + (o.kind == Op::kAllGather ? (size_t)p * o.bytes : 0);
            if (o.bytes && hipMemcpy(dst, in[p].data() + at[p], o.bytes, hipMemcpyHostToDevice) != hipSuccess)
                return ncclUnhandledCudaError;
            at[p] += o.bytes;
        }
    }
    return ncclSuccess;
}

ncclResult_t enqueue(const Op &o)
{
    g_ops.push_back(o);
    if (g_depth > 0)
        return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    return run(ops);
}
}  // namespace

extern "C"
{
ncclResult_t ncclGetUniqueId(ncclUniqueId *id)
{
    char tmpl[] = "/tmp/cwf_host_nccl.XXXXXX";
    if (!mkdtemp(tmpl))
        return ncclSystemError;
    memset(id, 0, sizeof *id);
    snprintf(id->internal, sizeof id->internal, "%s", tmpl);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank)
{
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return ncclInvalidArgument;
    auto *c = new HostComm;
    c->n = nranks;
    c->rank = rank;
    c->dir = id.internal;
    c->fd.assign(nranks, -1);
    c->listen_fd = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un me = addr_of(c->dir, rank);
    unlink(me.sun_path);
    if (c->listen_fd < 0 || bind(c->listen_fd, reinterpret_cast<sockaddr *>(&me), sizeof me) != 0 ||
        listen(c->listen_fd, nranks) != 0)
        return ncclSystemError;
    for (int p = 0; p < rank; ++p)  // connect to the lower ranks (retrying until they listen), say who we are
    {
        const sockaddr_un a = addr_of(c->dir, p);
        int fd = -1;
        for (int t = 0; t < 6000 && fd < 0; ++t)
        {
            fd = socket(AF_UNIX, SOCK_STREAM, 0);
            if (connect(fd, reinterpret_cast<const sockaddr *>(&a), sizeof a) != 0)
            {
                close(fd);
                fd = -1;
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            }
        }
        if (fd < 0 || !write_all(fd, &rank, sizeof rank))
            return ncclSystemError;
        c->fd[p] = fd;
    }
    for (int k = rank + 1; k < nranks; ++k)  // accept the higher ranks
    {
        const int fd = accept(c->listen_fd, nullptr, nullptr);
        int who = -1;
        if (fd < 0 || !read_all(fd, &who, sizeof who) || who <= rank || who >= nranks)
            return ncclSystemError;
        c->fd[who] = fd;
    }
    *comm = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm)
{
    auto *c = reinterpret_cast<HostComm *>(comm);
    if (!c)
        return ncclSuccess;
    for (int fd : c->fd)
        if (fd >= 0)
            close(fd);
    if (c->listen_fd >= 0)
        close(c->listen_fd);
    const sockaddr_un me = addr_of(c->dir, c->rank);
    unlink(me.sun_path);
    if (c->rank == 0)
        rmdir(c->dir.c_str());  // succeeds once the last socket file is gone
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t stream)
{
    const size_t b = type_bytes(t);
    if (!b || !comm)
        return ncclInvalidArgument;
    return enqueue({Op::kAllGather, sendbuff, recvbuff, count * b, -1, reinterpret_cast<HostComm *>(comm), stream});
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                      hipStream_t stream)
{
    auto *c = reinterpret_cast<HostComm *>(comm);
    const size_t b = type_bytes(t);
    if (!b || !c || peer < 0 || peer >= c->n || peer == c->rank)
        return ncclInvalidArgument;
    return enqueue({Op::kSend, sendbuff, nullptr, count * b, peer, c, stream});
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t stream)
{
    auto *c = reinterpret_cast<HostComm *>(comm);
    const size_t b = type_bytes(t);
    if (!b || !c || peer < 0 || peer >= c->n || peer == c->rank)
        return ncclInvalidArgument;
    return enqueue({Op::kRecv, nullptr, recvbuff, count * b, peer, c, stream});
}

ncclResult_t ncclGroupStart()
{
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd()
{
    if (g_depth <= 0)
        return ncclInvalidUsage;
    if (--g_depth > 0)
        return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    return run(ops);
}

const char *ncclGetErrorString(ncclResult_t r)
{
    switch (r)
    {
    case ncclSuccess:
        return "no error";
    case ncclUnhandledCudaError:
        return "host transport: HIP call failed";
    case ncclSystemError:
        return "host transport: socket error";
    case ncclInvalidArgument:
        return "host transport: invalid argument";
    case ncclInvalidUsage:
        return "host transport: invalid usage";
    default:
        return "host transport: error";
    }
}
}
