/* rccl_shim.c -- test stand-in for the four RCCL entry points that
 * srtp_mi355x_session_broadcast resolves at run time (ncclBroadcast,
 * ncclAllReduce, ncclCommUserRank, ncclGetErrorString), for two ranks in
 * two processes on ONE GPU, where RCCL itself refuses to run.  The bytes
 * move between the processes over a Unix stream socket: device buffer ->
 * host (hipMemcpy) -> socket -> host -> device buffer.  Loaded with
 * RTLD_GLOBAL by tests/bcast_rank.py so the library's dlsym(RTLD_DEFAULT)
 * finds it; the product library never links it.  Test infrastructure only.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

typedef struct {
    int rank, nranks, fd;
} shim_comm_t;

static int io_all(int fd, void *p, size_t n, int wr)
{
    uint8_t *b = (uint8_t *)p;
    while (n) {
        ssize_t k = wr ? write(fd, b, n) : read(fd, b, n);
        if (k <= 0)
            return -1;
        b += k;
        n -= (size_t)k;
    }
    return 0;
}

/* rank 0 listens on `path`, rank 1 connects (retrying for ~10 s) */
void *shim_comm_init(int rank, int nranks, const char *path)
{
    if (nranks != 2 || rank < 0 || rank > 1)
        return NULL;
    shim_comm_t *c = (shim_comm_t *)calloc(1, sizeof *c);
    struct sockaddr_un a;
    memset(&a, 0, sizeof a);
    a.sun_family = AF_UNIX;
    strncpy(a.sun_path, path, sizeof a.sun_path - 1);
    int s = socket(AF_UNIX, SOCK_STREAM, 0);
    if (!c || s < 0)
        return NULL;
    if (rank == 0) {
        unlink(path);
        if (bind(s, (struct sockaddr *)&a, sizeof a) || listen(s, 1))
            return NULL;
        c->fd = accept(s, NULL, NULL);
        close(s);
    } else {
        int ok = -1;
        for (int t = 0; t < 1000 && ok; t++) {
            ok = connect(s, (struct sockaddr *)&a, sizeof a);
            if (ok)
                usleep(10000);
        }
        if (ok)
            return NULL;
        c->fd = s;
    }
    c->rank = rank;
    c->nranks = nranks;
    return c->fd < 0 ? NULL : c;
}

void shim_comm_free(void *comm)
{
    shim_comm_t *c = (shim_comm_t *)comm;
    if (c) {
        close(c->fd);
        free(c);
    }
}

static size_t type_size(int t)
{
    /* rccl.h ncclDataType_t: int8 0, uint8 1, int32 2, uint32 3, int64 4,
     * uint64 5 */
    return t <= 1 ? 1 : t <= 3 ? 4 : 8;
}

int ncclCommUserRank(void *comm, int *rank)
{
    if (!comm)
        return 4;   /* ncclInvalidArgument */
    *rank = ((shim_comm_t *)comm)->rank;
    return 0;
}

const char *ncclGetErrorString(int r)
{
    return r ? "rccl_shim: error" : "no error";
}

int ncclBroadcast(const void *send, void *recv, size_t count, int dtype,
                  int root, void *comm, hipStream_t stream)
{
    shim_comm_t *c = (shim_comm_t *)comm;
    const size_t n = count * type_size(dtype);
    uint8_t *h = (uint8_t *)malloc(n ? n : 1);
    if (!c || !h || hipStreamSynchronize(stream) != hipSuccess)
        return 2;   /* ncclSystemError */
    int rc = 0;
    if (c->rank == root) {
        if (hipMemcpy(h, send, n, hipMemcpyDeviceToHost) != hipSuccess ||
            io_all(c->fd, h, n, 1) ||
            (recv != send &&
             hipMemcpy(recv, send, n, hipMemcpyDeviceToDevice) != hipSuccess))
            rc = 2;
    } else if (io_all(c->fd, h, n, 0) ||
               hipMemcpy(recv, h, n, hipMemcpyHostToDevice) != hipSuccess) {
        rc = 2;
    }
    free(h);
    return rc;
}

/* uint64 sum (op 0) / max (op 2) over the two ranks */
int ncclAllReduce(const void *send, void *recv, size_t count, int dtype,
                  int op, void *comm, hipStream_t stream)
{
    shim_comm_t *c = (shim_comm_t *)comm;
    if (!c || dtype != 5 || (op != 0 && op != 2))
        return 4;
    const size_t n = count * 8;
    uint64_t *a = (uint64_t *)malloc(n ? n : 8), *b = (uint64_t *)malloc(n ? n : 8);
    int rc = 0;
    if (!a || !b || hipStreamSynchronize(stream) != hipSuccess ||
        hipMemcpy(a, send, n, hipMemcpyDeviceToHost) != hipSuccess) {
        rc = 2;
    } else if (c->rank == 0 ? (io_all(c->fd, a, n, 1) || io_all(c->fd, b, n, 0))
                            : (io_all(c->fd, b, n, 0) || io_all(c->fd, a, n, 1))) {
        rc = 2;
    } else {
        for (size_t k = 0; k < count; k++)
            a[k] = op == 0 ? a[k] + b[k] : (a[k] > b[k] ? a[k] : b[k]);
        if (hipMemcpy(recv, a, n, hipMemcpyHostToDevice) != hipSuccess)
            rc = 2;
    }
    free(a);
    free(b);
    return rc;
}
