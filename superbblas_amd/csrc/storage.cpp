// Tensor storage in the S3T file format of superbblas (storage.h): create / open / append
// blocks / save / load / get_blocks / checksums / close.
//
// Reference: the format specification at storage.h:19-54; create_storage 1432-1520,
// open_storage 1535-1625, append_blocks 1680-1800, read_all_blocks 1805-1880, save 1198-1315,
// load 1326-1385, get_blocks 1396-1420, check_or_write_checksums 1935-2125, do_checksum
// 700-735 (zlib CRC-32; above checksum_blocksize: CRC of the per-chunk CRCs).
//  * Files are read and written with POSIX pread/pwrite at explicit offsets, so every rank of a
//    communicator writes its own pieces of a shared file concurrently; rank 0 writes the headers
//    and the checksums, and the ranks meet at barriers around the collective steps.
//  * save: each (component piece x stored block) box is packed on the GPU into the block's order
//    with the element conversion and alpha fused (the library's box copy), brought to the host in
//    one transfer and written as the contiguous runs of the block; load is the reverse (read the
//    runs, one upload, one box copy into the component).
//  * Block lookups scan the stored blocks in append order (the reference's GridHash visits them
//    in grid order): the bytes of a file are the reference's as long as a new block overlaps at
//    most one stored block (otherwise the same elements are stored, possibly split differently),
//    and get_blocks may list the same boxes in another order.
#include "plan.h"

#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstring>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

namespace sbx {

// ---------------------------------------------------------------------------------------------
// CRC-32 (the zlib / IEEE 802.3 polynomial, reflected 0xEDB88320), table driven
// ---------------------------------------------------------------------------------------------
namespace {

struct CrcTable {
    uint32_t t[256];
    CrcTable() {
        for (uint32_t n = 0; n < 256; ++n) {
            uint32_t c = n;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[n] = c;
        }
    }
};

uint32_t crc32_update(uint32_t crc, const void *buf, std::size_t len) {
    static const CrcTable tab;
    const unsigned char *p = (const unsigned char *)buf;
    crc = ~crc;
    for (std::size_t i = 0; i < len; ++i) crc = tab.t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}

/// storage.h:709-735: plain CRC, or (blocksize > 0) the CRC of the CRCs of blocksize chunks
uint32_t do_checksum(const void *p, std::size_t bytes, std::size_t blocksize = 0,
                     uint32_t prev = 0) {
    if (blocksize == 0) return crc32_update(prev, p, bytes);
    if (prev != 0) throw Error("Ups! This should not happen");
    const std::size_t nb = (bytes + blocksize - 1) / blocksize;
    std::vector<uint32_t> cs(nb);
    for (std::size_t i = 0; i < nb; ++i)
        cs[i] = crc32_update(0, (const char *)p + i * blocksize, std::min(blocksize, bytes - i * blocksize));
    return crc32_update(0, cs.data(), nb * sizeof(uint32_t));
}

constexpr int MAGIC = 314;
constexpr std::size_t DEFAULT_CHECKSUM_BLOCKSIZE = 64u * 1024 * 1024;

[[noreturn]] void io_error(const std::string &what) {
    throw Error(what + ": " + std::strerror(errno));
}

void pwrite_all(int fd, const void *buf, std::size_t n, std::size_t off) {
    const char *p = (const char *)buf;
    while (n > 0) {
        const ssize_t w = ::pwrite(fd, p, n, (off_t)off);
        if (w < 0) {
            if (errno == EINTR) continue;
            io_error("Error writing in a file");
        }
        p += w;
        n -= (std::size_t)w;
        off += (std::size_t)w;
    }
}

void pread_all(int fd, void *buf, std::size_t n, std::size_t off) {
    char *p = (char *)buf;
    while (n > 0) {
        const ssize_t r = ::pread(fd, p, n, (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            io_error("Error reading from a file");
        }
        if (r == 0) {
            errno = 0;
            throw Error("Error reading from a file: unexpected end of file");
        }
        p += r;
        n -= (std::size_t)r;
        off += (std::size_t)r;
    }
}

void swap_bytes(void *p, std::size_t n, std::size_t width) {
    char *c = (char *)p;
    for (std::size_t i = 0; i < n; ++i, c += width)
        for (std::size_t j = 0; j < width / 2; ++j) std::swap(c[j], c[width - 1 - j]);
}

/// values_datatype (storage.h:63) <-> the ABI's element types (CHAR has no ABI type here)
int vtype_of(int dtype) {
    switch (dtype) {
    case SBX_FLOAT: return 0;
    case SBX_DOUBLE: return 1;
    case SBX_CFLOAT: return 2;
    case SBX_CDOUBLE: return 3;
    case SBX_INT: return 5;
    }
    throw Error("storage: unsupported type");
}
int dtype_of_vtype(int v) {
    switch (v) {
    case 0: return SBX_FLOAT;
    case 1: return SBX_DOUBLE;
    case 2: return SBX_CFLOAT;
    case 3: return SBX_CDOUBLE;
    case 5: return SBX_INT;
    }
    throw Error("storage: unsupported values datatype in the file");
}
/// width of the scalars to byte swap for a type (complex: the real type)
std::size_t scalar_width(int dtype) {
    return dtype_is_complex(dtype) ? dtype_size(dtype) / 2 : dtype_size(dtype);
}

} // namespace

/// the checksum of the S3T format (storage.h:701-731) for detail::do_checksum (sbx_checksum)
uint32_t storage_checksum(const void *p, std::size_t bytes, std::size_t blocksize, uint32_t prev) {
    return do_checksum(p, bytes, blocksize, prev);
}

struct StorageCtx {
    int fd = -1;
    int dtype = SBX_CDOUBLE; // element type of the values
    Coor dim;                // SlowToFast
    std::size_t header_size = 0, disp = 0;
    bool swap = false;
    int checksum = 0;
    std::size_t blocksize = DEFAULT_CHECKSUM_BLOCKSIZE;
    uint32_t checksum_val = 0;
    std::size_t num_chunks = 0;
    bool allow_writing = false, modified_flush = false, modified_checksum = false;
    std::vector<Range> blocks;
    std::vector<std::size_t> disp_values, disp_checksum;
    std::vector<char> checksum_done;
    int nprocs = 1, rank = 0;

    std::size_t es() const { return dtype_size(dtype); }
    ~StorageCtx() {
        if (fd >= 0) {
            if (allow_writing && rank == 0)
                (void)::ftruncate(fd, (off_t)(disp + (checksum == 0 ? 0 : sizeof(double))));
            ::close(fd);
        }
    }

    /// stored blocks overlapping [from, from+size): (block index, range relative to the block)
    std::vector<std::pair<std::size_t, Range>> overlaps(const Range &q) const {
        std::vector<std::pair<std::size_t, Range>> r;
        if (volume(q.size) == 0) return r;
        for (std::size_t b = 0; b < blocks.size(); ++b)
            for (const Range &x : intersection(blocks[b], q, dim)) {
                if (volume(x.size) == 0) continue;
                Range rel{Coor(dim.size()), x.size};
                for (std::size_t i = 0; i < dim.size(); ++i)
                    rel.from[i] = normalize_coor((long)x.from[i] - blocks[b].from[i], dim[i]);
                r.push_back({b, rel});
            }
        return r;
    }

    void add_block(const Range &b, std::size_t values_disp) {
        // GridHash::append_block normalises `from` of whole dimensions (storage.h:577-584)
        Range n = b;
        for (std::size_t i = 0; i < dim.size(); ++i)
            n.from[i] = n.size[i] == dim[i] ? 0 : normalize_coor(n.from[i], dim[i]);
        blocks.push_back(n);
        disp_values.push_back(values_disp);
    }
};

namespace {

/// The header's fixed part (storage.h:1456-1509): returns its bytes and the running checksum
std::string header_bytes(int vtype, int checksum, const Coor &dim, const char *meta, int len) {
    std::string h;
    auto put = [&](const void *p, std::size_t n) { h.append((const char *)p, n); };
    const int ints[5] = {MAGIC, 0, vtype, checksum, (int)dim.size()};
    put(ints, sizeof(ints));
    put(&len, sizeof(int));
    put(meta, (std::size_t)len);
    const std::string pad((8 - len % 8) % 8, '\0');
    put(pad.data(), pad.size());
    for (int d : dim) {
        const double x = d;
        put(&x, sizeof(double));
    }
    const double bs = (double)DEFAULT_CHECKSUM_BLOCKSIZE;
    put(&bs, sizeof(double));
    return h;
}

/// read the header (storage.h:1535-1625); dims SlowToFast as stored
void read_header(int fd, int &vtype, std::string &meta, Coor &dim, std::size_t &header_size,
                 bool &swap, int &checksum, std::size_t &blocksize, uint32_t &checksum_val) {
    std::size_t off = 0;
    auto rd = [&](void *p, std::size_t n) {
        pread_all(fd, p, n, off);
        off += n;
    };
    int i32;
    rd(&i32, 4);
    swap = false;
    if (i32 != MAGIC) {
        swap_bytes(&i32, 1, 4);
        if (i32 != MAGIC)
            throw Error("Unexpected value for the magic number; the file may not be a tensor "
                        "storage");
        swap = true;
    }
    auto rdi = [&]() {
        int v;
        rd(&v, 4);
        if (swap) swap_bytes(&v, 1, 4);
        return v;
    };
    if (rdi() != 0)
        throw Error("Unsupported version of the tensor format; try a newer version of supperbblas");
    vtype = rdi();
    checksum = rdi();
    if (checksum < 0 || checksum > 2) throw Error("Unsupported checksum type");
    const int nd = rdi();
    const int len = rdi();
    if (nd < 0 || len < 0) throw Error("storage: corrupted header");
    meta.assign((std::size_t)len, '\0');
    if (len) rd(&meta[0], (std::size_t)len);
    off += (8 - len % 8) % 8;
    std::vector<double> d(nd);
    if (nd) rd(d.data(), sizeof(double) * nd);
    if (swap) swap_bytes(d.data(), nd, 8);
    dim.assign(nd, 0);
    for (int i = 0; i < nd; ++i) dim[i] = (int)d[i];
    double bs;
    rd(&bs, 8);
    if (swap) swap_bytes(&bs, 1, 8);
    blocksize = (std::size_t)bs;
    header_size = sizeof(int) * 6 + len + (8 - len % 8) % 8 + sizeof(double) * (nd + 1);
    checksum_val = 0;
    if (checksum == 2) {
        std::string h(header_size, '\0');
        pread_all(fd, &h[0], header_size, 0);
        checksum_val = do_checksum(h.data(), header_size);
    }
}

/// read_all_blocks (storage.h:1805-1880)
void read_all_blocks(StorageCtx &s) {
    std::size_t cur = s.header_size;
    double nc;
    pread_all(s.fd, &nc, 8, cur);
    cur += 8;
    if (s.swap) swap_bytes(&nc, 1, 8);
    s.num_chunks = (std::size_t)nc;
    const int nd = (int)s.dim.size();
    for (std::size_t chunk = 0; chunk < s.num_chunks; ++chunk) {
        double d;
        pread_all(s.fd, &d, 8, cur);
        if (s.checksum == 2) s.checksum_val = do_checksum(&d, 8, 0, s.checksum_val);
        if (s.swap) swap_bytes(&d, 1, 8);
        const std::size_t nb = (std::size_t)d;
        std::vector<double> fs(nb * 2 * nd);
        if (nb) pread_all(s.fd, fs.data(), fs.size() * 8, cur + 8);
        if (s.checksum == 2 && nb) s.checksum_val = do_checksum(fs.data(), fs.size() * 8, 0, s.checksum_val);
        if (s.swap) swap_bytes(fs.data(), fs.size(), 8);
        cur += 8 + nb * nd * 16;
        for (std::size_t i = 0; i < nb; ++i) {
            Range b{Coor(nd), Coor(nd)};
            for (int k = 0; k < nd; ++k) {
                b.from[k] = (int)fs[(i * 2) * nd + k];
                b.size[k] = (int)fs[(i * 2 + 1) * nd + k];
            }
            s.add_block(b, cur);
            cur += volume(b.size) * s.es();
        }
        if (s.checksum == 2)
            for (std::size_t i = 0; i < nb; ++i) {
                s.disp_checksum.push_back(cur);
                s.checksum_done.push_back(1);
                cur += 8;
            }
    }
    s.disp = cur;
    if (s.checksum != 0) {
        double d;
        pread_all(s.fd, &d, 8, cur);
        if (s.swap) swap_bytes(&d, 1, 8);
        if (s.checksum == 2 && (double)s.checksum_val != d) throw Error("Checksum failed!");
        if (s.checksum == 1) s.checksum_val = (uint32_t)d;
    }
}

int open_fd(const char *filename, int flags) {
    const int fd = ::open(filename, flags, 0644);
    if (fd < 0) io_error(std::string("Error opening file `") + filename + "'");
    return fd;
}

/// Contiguous runs of a sub-box [rel, rel+size) of a dense SlowToFast array of dims `bdim`:
/// calls f(element offset in the array, offset in the dense sub-box, run length)
template <typename F> void for_runs(const Coor &rel, const Coor &size, const Coor &bdim, F &&f) {
    const int nd = (int)bdim.size();
    const std::vector<long> st = strides_slow_to_fast(bdim);
    // merge the fastest dims that the sub-box covers whole (get_normalize_permutation)
    long run = 1;
    int k = nd - 1;
    for (; k >= 0; --k) {
        run *= size[k];
        if (rel[k] != 0 || size[k] != bdim[k]) {
            --k;
            break;
        }
    }
    // dims 0..k are iterated
    const long nrun = volume(size) / std::max(1L, run);
    Coor c(nd, 0);
    for (long r = 0; r < nrun; ++r) {
        long off = 0, rem = r;
        for (int i = k; i >= 0; --i) {
            c[i] = (int)(rem % size[i]);
            rem /= size[i];
        }
        for (int i = 0; i < nd; ++i) off += (long)(rel[i] + (i <= k ? c[i] : 0)) * st[i];
        f(off, r * run, run);
    }
}

} // namespace

// ---------------------------------------------------------------------------------------------
// API
// ---------------------------------------------------------------------------------------------

StorageCtx *storage_create(int dtype, const Coor &dim, const char *filename, const char *meta,
                           int meta_len, int checksum, const Comm &comm) {
    if (checksum < 0 || checksum > 2) throw Error("storage: invalid checksum type");
    if (meta_len < 0 || (meta_len > 0 && !meta)) throw Error("storage: invalid metadata");
    std::unique_ptr<StorageCtx> s(new StorageCtx());
    s->dtype = dtype;
    s->dim = dim;
    s->checksum = checksum;
    s->nprocs = comm.nprocs;
    s->rank = comm.rank;
    s->allow_writing = true;
    s->modified_flush = s->modified_checksum = true;
    const std::string h = header_bytes(vtype_of(dtype), checksum, dim, meta ? meta : "", meta_len);
    s->header_size = h.size();
    s->checksum_val = do_checksum(h.data(), h.size());
    if (comm.rank == 0) {
        s->fd = open_fd(filename, O_RDWR | O_CREAT | O_TRUNC);
        pwrite_all(s->fd, h.data(), h.size(), 0);
        const double zero = 0;
        pwrite_all(s->fd, &zero, 8, h.size());
    }
    comm_barrier(comm);
    if (comm.rank != 0) s->fd = open_fd(filename, O_RDWR);
    s->disp = s->header_size + 8;
    return s.release();
}

void storage_read_header(const char *filename, int &dtype, std::string &meta, Coor &dim) {
    const int fd = open_fd(filename, O_RDONLY);
    try {
        int vtype, checksum;
        std::size_t hs, bs;
        bool swap;
        uint32_t cv;
        read_header(fd, vtype, meta, dim, hs, swap, checksum, bs, cv);
        dtype = dtype_of_vtype(vtype);
    } catch (...) {
        ::close(fd);
        throw;
    }
    ::close(fd);
}

StorageCtx *storage_open(int nd, int dtype, const char *filename, bool allow_writing,
                         const Comm &comm) {
    std::unique_ptr<StorageCtx> s(new StorageCtx());
    s->nprocs = comm.nprocs;
    s->rank = comm.rank;
    s->fd = open_fd(filename, allow_writing ? O_RDWR : O_RDONLY);
    s->allow_writing = allow_writing;
    int vtype;
    std::string meta;
    read_header(s->fd, vtype, meta, s->dim, s->header_size, s->swap, s->checksum, s->blocksize,
                s->checksum_val);
    if (dtype_of_vtype(vtype) != dtype)
        throw Error("The template parameter T does not match with the datatype of the storage");
    if ((int)s->dim.size() != nd)
        throw Error("The template parameter Nd does not match with the number of dimensions of "
                    "the storage");
    s->dtype = dtype;
    read_all_blocks(*s);
    return s.release();
}

void storage_append_blocks(StorageCtx &s, const std::vector<Range> &p0, const std::string &o0,
                           const Coor &from0, const Coor &size0, const Coor &dim0,
                           const std::string &o1, const Coor &from1, const Comm &comm) {
    if (!s.allow_writing) throw Error("storage: opened read-only");
    const int nd = (int)s.dim.size();
    const Range region{from0, size0};
    std::vector<Range> new_blocks;
    std::vector<double> chunk(1);
    for (const Range &b : p0) {
        // restrict to the region (a single box, dist.h:436-451) and translate to the storage
        std::vector<Range> ri = intersection(region, b, dim0);
        if (ri.size() > 1) throw Error("Not supported complex overlap of intervals");
        Range t{Coor(nd, 0), Coor(nd, 0)};
        if (!ri.empty() && volume(ri[0].size) > 0) t = translate(ri[0], o0, from0, dim0, o1, from1, s.dim);
        // remove what is already stored; as the reference (storage.h:1725-1730) both the stored
        // block and the intersection range it reports (relative to that block) are removed
        std::vector<Range> holes;
        for (const auto &o : s.overlaps(t)) {
            holes.push_back(s.blocks[o.first]);
            holes.push_back(o.second);
        }
        std::vector<Range> fs(1, t);
        if (volume(t.size) == 0) fs.clear();
        for (const std::vector<Range> *hs : {&holes, &new_blocks})
            for (const Range &h : *hs) {
                std::vector<Range> nfs;
                for (const Range &r : fs)
                    for (const Range &q : make_hole(r, h, s.dim))
                        if (volume(q.size) > 0) nfs.push_back(q);
                fs.swap(nfs);
            }
        for (const Range &r : fs) {
            new_blocks.push_back(r);
            chunk.insert(chunk.end(), r.from.begin(), r.from.end());
            chunk.insert(chunk.end(), r.size.begin(), r.size.end());
        }
    }
    if (new_blocks.empty()) return;
    std::size_t values = s.disp + 8 + new_blocks.size() * nd * 16;
    for (const Range &r : new_blocks) {
        s.add_block(r, values);
        values += volume(r.size) * s.es();
    }
    chunk[0] = (double)new_blocks.size();
    if (s.swap) swap_bytes(chunk.data(), chunk.size(), 8);
    if (s.checksum == 2) s.checksum_val = do_checksum(chunk.data(), chunk.size() * 8, 0, s.checksum_val);
    if (comm.rank == 0) pwrite_all(s.fd, chunk.data(), chunk.size() * 8, s.disp);
    if (s.checksum == 2)
        for (std::size_t i = 0; i < new_blocks.size(); ++i) {
            s.disp_checksum.push_back(values);
            s.checksum_done.push_back(0);
            values += 8;
        }
    s.disp = values;
    s.num_chunks++;
    if (comm.rank == 0) {
        double n = (double)s.num_chunks;
        if (s.swap) swap_bytes(&n, 1, 8);
        pwrite_all(s.fd, &n, 8, s.header_size);
    }
    s.modified_flush = s.modified_checksum = true;
}

namespace {
/// one piece to move between a tensor and a stored block
struct Op {
    int comp;       // index of the tensor range it came from
    Range in_comp;  // box in absolute tensor coordinates (tensor labels)
    std::size_t b;  // block
    Range in_block; // box relative to the block (storage labels, SlowToFast)
};

/// Pieces of tensor ranges (tensor labels lt, dims dimt, region [fromt, fromt+sizet))
/// against the stored blocks (storage_labels, region start froms) -- get_overlap_ranges,
/// storage.h:844-890
std::vector<Op> overlap_ops(const StorageCtx &s, const std::vector<Range> &comps,
                            const std::vector<int> &comp_ids, const std::string &lt,
                            const Coor &dimt, const Coor &fromt, const Coor &sizet,
                            const std::string &ls, const Coor &froms) {
    std::vector<Op> ops;
    for (std::size_t i = 0; i < comps.size(); ++i) {
        std::vector<Range> ri = intersection(Range{fromt, sizet}, comps[i], dimt);
        if (ri.size() > 1) throw Error("Not supported complex overlap of intervals");
        if (ri.empty() || volume(ri[0].size) == 0) continue;
        const Range t = translate(ri[0], lt, fromt, dimt, ls, froms, s.dim);
        for (const auto &o : s.overlaps(t)) {
            Range abs{Coor(s.dim.size()), o.second.size};
            for (std::size_t k = 0; k < s.dim.size(); ++k)
                abs.from[k] = normalize_coor((long)s.blocks[o.first].from[k] + o.second.from[k], s.dim[k]);
            ops.push_back({comp_ids[i], translate(abs, ls, froms, s.dim, lt, fromt, dimt), o.first,
                           o.second});
        }
    }
    return ops;
}

/// Split a piece whose box runs past the end of its component or block (possible when that
/// component or block spans a whole periodic dimension; the reference's local copies wrap
/// there, storage.h:895-939) into pieces that do not wrap
void split_wraps(const Op &op, const Coor &comp_size, const Coor &block_size,
                 const std::string &lt, const Coor &dimt, const std::string &ls,
                 const Coor &dims, std::vector<Op> &out) {
    for (std::size_t k = 0; k < lt.size(); ++k) {
        const long c = op.in_comp.from[k], n = op.in_comp.size[k], L = comp_size[k];
        if (c + n <= L) continue;
        const int first = (int)(L - c);
        Op a = op, b = op;
        a.in_comp.size[k] = first;
        b.in_comp.from[k] = 0;
        b.in_comp.size[k] = (int)(n - first);
        const auto j = ls.find(lt[k]);
        if (j != std::string::npos) {
            a.in_block.size[j] = first;
            b.in_block.from[j] = normalize_coor((long)op.in_block.from[j] + first, dims[j]);
            b.in_block.size[j] = (int)(n - first);
        }
        split_wraps(a, comp_size, block_size, lt, dimt, ls, dims, out);
        split_wraps(b, comp_size, block_size, lt, dimt, ls, dims, out);
        return;
    }
    for (std::size_t j = 0; j < ls.size(); ++j) {
        const long c = op.in_block.from[j], n = op.in_block.size[j], L = block_size[j];
        if (c + n <= L) continue;
        const int first = (int)(L - c);
        Op a = op, b = op;
        a.in_block.size[j] = first;
        b.in_block.from[j] = 0;
        b.in_block.size[j] = (int)(n - first);
        const auto k = lt.find(ls[j]);
        if (k != std::string::npos) {
            a.in_comp.size[k] = first;
            b.in_comp.from[k] = normalize_coor((long)op.in_comp.from[k] + first, dimt[k]);
            b.in_comp.size[k] = (int)(n - first);
        }
        split_wraps(a, comp_size, block_size, lt, dimt, ls, dims, out);
        split_wraps(b, comp_size, block_size, lt, dimt, ls, dims, out);
        return;
    }
    out.push_back(op);
}

std::vector<long> strides_of(const Coor &size) { return strides_slow_to_fast(size); }

/// box copy: src (labels ls, dense dims ssize) at sfrom -> dst (labels ld, dense dims dsize) at
/// dfrom, `box` in source labels
void box_copy(const Scalar &alpha, int st, const void *src, const std::string &ls,
              const Coor &ssize, const Coor &sfrom, int dt, void *dst, const std::string &ld,
              const Coor &dsize, const Coor &dfrom, const Coor &box, int device) {
    const std::vector<long> ss = strides_of(ssize), ds = strides_of(dsize);
    BoxCopyDesc d;
    d.src_t = st;
    d.dst_t = dt;
    long so = 0, doff = 0;
    for (std::size_t k = 0; k < ls.size(); ++k) so += (long)sfrom[k] * ss[k];
    for (std::size_t k = 0; k < ld.size(); ++k) doff += (long)dfrom[k] * ds[k];
    d.src = (const char *)src + so * dtype_size(st);
    d.dst = (char *)dst + doff * dtype_size(dt);
    d.size.assign(box.begin(), box.end());
    d.src_stride = ss;
    d.dst_stride.resize(ls.size());
    for (std::size_t k = 0; k < ls.size(); ++k) {
        const auto j = ld.find(ls[k]);
        d.dst_stride[k] = j == std::string::npos ? 0 : ds[j];
    }
    d.alpha = alpha;
    d.add = false;
    launch_box_copy(d, device);
}
} // namespace

void storage_save(StorageCtx &s, const Scalar &alpha, const DistTensor &v, const Coor &from0,
                  const Coor &size0, const std::string &o1, const Coor &from1, const Comm &comm) {
    if (!s.allow_writing) throw Error("storage: opened read-only");
    const int nd = (int)s.dim.size();
    if ((int)o1.size() != nd) throw Error("storage: invalid storage labels");
    // ranges to save: remove overlaps with earlier components of the rank and with lower
    // ranks (storage.h:1230-1250); all ranks are visited for the block-checksum bookkeeping
    std::vector<Op> mine;
    for (int rk = 0; rk < comm.nprocs; ++rk) {
        if (s.checksum != 2 && rk != comm.rank) continue;
        std::vector<Range> done;
        for (int c = 0; c < (int)v.ranges[rk].size(); ++c) {
            std::vector<Range> rs;
            if (volume(v.ranges[rk][c].size) > 0) rs.push_back(v.ranges[rk][c]);
            auto cut = [&](const std::vector<Range> &holes) {
                for (const Range &h : holes) {
                    if (volume(h.size) == 0) continue;
                    std::vector<Range> n;
                    for (const Range &r : rs)
                        for (const Range &q : make_hole(r, h, v.dim))
                            if (volume(q.size) > 0) n.push_back(q);
                    rs.swap(n);
                }
            };
            cut(done);
            for (int r = 0; r < rk; ++r) cut(v.ranges[r]);
            done.insert(done.end(), rs.begin(), rs.end());
            std::vector<int> ids(rs.size(), c);
            std::vector<Op> pieces;
            for (Op op : overlap_ops(s, rs, ids, v.labels, v.dim, from0, size0, o1, from1)) {
                // relative to the component (storage.h:1270-1275)
                for (int k = 0; k < v.nd(); ++k)
                    op.in_comp.from[k] = normalize_coor(
                        (long)op.in_comp.from[k] - v.ranges[rk][c].from[k], v.dim[k]);
                split_wraps(op, v.ranges[rk][c].size, s.blocks[op.b].size, v.labels, v.dim, o1,
                            s.dim, pieces);
            }
            // a block wholly written by one piece gets its checksum on the fly (storage.h:1256-
            // 1266, 1048-1055); every rank tracks which, for the checksums written at close
            if (s.checksum == 2)
                for (const Op &op : pieces)
                    s.checksum_done[op.b] = (op.in_block.from == Coor(nd, 0) &&
                                             op.in_block.size == s.blocks[op.b].size)
                                                ? 1
                                                : 0;
            if (rk == comm.rank) mine.insert(mine.end(), pieces.begin(), pieces.end());
        }
    }
    const std::size_t es = s.es();
    for (const Op &op : mine) {
        const int dev = v.dev[op.comp];
        const Range &cr = v.ranges[comm.rank][op.comp];
        // translate the piece box from component-relative to the storage order
        const long n = volume(op.in_block.size);
        Scratch dbuf(n * es, dev);
        Coor box(v.nd());
        for (int k = 0; k < v.nd(); ++k) box[k] = op.in_comp.size[k];
        box_copy(alpha, v.dtype, v.ptr[op.comp], v.labels, cr.size, op.in_comp.from, s.dtype,
                 dbuf.ptr, o1, op.in_block.size, Coor(nd, 0), box, dev);
        std::vector<char> host(n * es);
        set_device(dev);
        SBX_HIP_CHECK(hipMemcpyAsync(host.data(), dbuf.ptr, n * es, hipMemcpyDeviceToHost,
                                     get_stream(dev)));
        SBX_HIP_CHECK(hipStreamSynchronize(get_stream(dev)));
        if (s.swap) swap_bytes(host.data(), n * es / scalar_width(s.dtype), scalar_width(s.dtype));
        const std::size_t base = s.disp_values[op.b];
        for_runs(op.in_block.from, op.in_block.size, s.blocks[op.b].size,
                 [&](long off, long pos, long run) {
                     pwrite_all(s.fd, host.data() + pos * es, run * es, base + off * es);
                 });
        if (s.checksum == 2 && op.in_block.from == Coor(nd, 0) &&
            op.in_block.size == s.blocks[op.b].size) {
            double c = do_checksum(host.data(), host.size(), s.blocksize);
            if (s.swap) swap_bytes(&c, 1, 8);
            pwrite_all(s.fd, &c, 8, s.disp_checksum[op.b]);
        }
    }
    s.modified_flush = s.modified_checksum = true;
}

void storage_load(StorageCtx &s, const Scalar &alpha, const std::string &o0, const Coor &from0,
                  const Coor &size0, const DistTensor &v, const Coor &from1, const Comm &comm) {
    const int nd = (int)s.dim.size();
    if ((int)o0.size() != nd) throw Error("storage: invalid storage labels");
    // region in the tensor's coordinates
    Coor size1(v.nd(), 1);
    for (int k = 0; k < v.nd(); ++k) {
        const auto j = o0.find(v.labels[k]);
        if (j != std::string::npos) size1[k] = size0[j];
    }
    std::vector<int> ids;
    for (int c = 0; c < (int)v.ranges[comm.rank].size(); ++c) ids.push_back(c);
    std::vector<Op> ops =
        overlap_ops(s, v.ranges[comm.rank], ids, v.labels, v.dim, from1, size1, o0, from0);
    const std::size_t es = s.es();
    std::vector<Op> pieces;
    for (Op &op : ops) {
        for (int k = 0; k < v.nd(); ++k)
            op.in_comp.from[k] = normalize_coor(
                (long)op.in_comp.from[k] - v.ranges[comm.rank][op.comp].from[k], v.dim[k]);
        split_wraps(op, v.ranges[comm.rank][op.comp].size, s.blocks[op.b].size, v.labels, v.dim,
                    o0, s.dim, pieces);
    }
    for (const Op &op : pieces) {
        const int dev = v.dev[op.comp];
        const long n = volume(op.in_block.size);
        std::vector<char> host(n * es);
        const std::size_t base = s.disp_values[op.b];
        for_runs(op.in_block.from, op.in_block.size, s.blocks[op.b].size,
                 [&](long off, long pos, long run) {
                     pread_all(s.fd, host.data() + pos * es, run * es, base + off * es);
                 });
        if (s.swap) swap_bytes(host.data(), n * es / scalar_width(s.dtype), scalar_width(s.dtype));
        Scratch dbuf(n * es, dev);
        set_device(dev);
        SBX_HIP_CHECK(hipMemcpyAsync(dbuf.ptr, host.data(), n * es, hipMemcpyHostToDevice,
                                     get_stream(dev)));
        // the values always replace the destination's (the reference's local_load copies,
        // storage.h:1160-1161, whatever CopyAdd was asked for)
        box_copy(alpha, s.dtype, dbuf.ptr, o0, op.in_block.size, Coor(nd, 0), v.dtype,
                 v.ptr[op.comp], v.labels, v.ranges[comm.rank][op.comp].size, op.in_comp.from,
                 op.in_block.size, dev);
        SBX_HIP_CHECK(hipStreamSynchronize(get_stream(dev)));
    }
}

std::vector<Range> storage_get_blocks(const StorageCtx &s, const std::string &o0,
                                      const std::string &o1, const Coor &from1,
                                      const Coor &size1) {
    // dims of the storage in o1's order, from0 = from1 reordered (storage.h:1405-1415)
    Coor dim1(o1.size(), 1), from0(o0.size(), 0);
    for (std::size_t k = 0; k < o1.size(); ++k) {
        const auto j = o0.find(o1[k]);
        if (j != std::string::npos) dim1[k] = s.dim[j];
    }
    for (std::size_t k = 0; k < o0.size(); ++k) {
        const auto j = o1.find(o0[k]);
        if (j != std::string::npos) from0[k] = from1[j];
    }
    std::vector<Range> out;
    std::vector<Op> ops = overlap_ops(s, std::vector<Range>(1, Range{from1, size1}),
                                      std::vector<int>(1, 0), o1, dim1, from1, size1, o0, from0);
    // relative to from1, as the reference reports them (storage.h:879, 1415-1418)
    for (const Op &op : ops) {
        Range r = op.in_comp;
        for (std::size_t k = 0; k < o1.size(); ++k)
            r.from[k] = normalize_coor((long)r.from[k] - from1[k], dim1[k]);
        out.push_back(r);
    }
    return out;
}

void storage_checksums(StorageCtx &s, const Comm &comm, bool do_write) {
    if (do_write && !s.modified_checksum) return;
    comm_barrier(comm);
    if (s.checksum == 1) {
        if (comm.rank == 0) {
            const std::size_t nb = (s.disp + s.blocksize - 1) / s.blocksize;
            std::vector<uint32_t> cs(nb);
            std::vector<char> buf(std::min(s.blocksize, s.disp));
            for (std::size_t b = 0; b < nb; ++b) {
                const std::size_t first = b * s.blocksize, n = std::min(s.disp - first, s.blocksize);
                pread_all(s.fd, buf.data(), n, first);
                cs[b] = do_checksum(buf.data(), n);
            }
            if (s.swap) swap_bytes(cs.data(), nb, 4);
            const uint32_t c = do_checksum(cs.data(), nb * 4);
            if (do_write) {
                s.checksum_val = c;
                double g = c;
                if (s.swap) swap_bytes(&g, 1, 8);
                pwrite_all(s.fd, &g, 8, s.disp);
            } else if (c != s.checksum_val) {
                throw Error("Checksum failed");
            }
        }
    } else if (s.checksum == 2) {
        if (comm.rank == 0) {
            std::vector<char> buf;
            for (std::size_t b = 0; b < s.blocks.size(); ++b) {
                if (do_write && s.checksum_done[b]) continue;
                const std::size_t n = volume(s.blocks[b].size) * s.es();
                if (n == 0) continue;
                buf.resize(n);
                pread_all(s.fd, buf.data(), n, s.disp_values[b]);
                double c = do_checksum(buf.data(), n, s.blocksize);
                if (do_write) {
                    if (s.swap) swap_bytes(&c, 1, 8);
                    pwrite_all(s.fd, &c, 8, s.disp_checksum[b]);
                } else {
                    double on_disk;
                    pread_all(s.fd, &on_disk, 8, s.disp_checksum[b]);
                    if (s.swap) swap_bytes(&on_disk, 1, 8);
                    if (c != on_disk)
                        throw Error("Checksum failed: block checksum failed on block " +
                                    std::to_string(b) + " : checksum " + std::to_string(on_disk) +
                                    " expected " + std::to_string(c));
                }
            }
            double h = s.checksum_val;
            if (do_write) {
                if (s.swap) swap_bytes(&h, 1, 8);
                pwrite_all(s.fd, &h, 8, s.disp);
            } else {
                double on_disk;
                pread_all(s.fd, &on_disk, 8, s.disp);
                if (s.swap) swap_bytes(&on_disk, 1, 8);
                if (on_disk != h) throw Error("Checksum failed: header checksum failed (postcheck)");
            }
        }
    }
    if (do_write) s.modified_checksum = false;
    comm_barrier(comm);
}

void storage_flush(StorageCtx &s) {
    if (s.fd >= 0 && ::fsync(s.fd) != 0 && errno != EINVAL) io_error("Error flushing file");
    s.modified_flush = false;
}

void storage_preallocate(StorageCtx &s, std::size_t size) {
    struct stat st;
    if (::fstat(s.fd, &st) != 0) io_error("Error getting the file size");
    if ((std::size_t)st.st_size < size && ::ftruncate(s.fd, (off_t)size) != 0)
        io_error("Error extending the file");
}

void storage_close(StorageCtx *s, const Comm &comm) {
    std::unique_ptr<StorageCtx> g(s);
    if (s->allow_writing) storage_checksums(*s, comm, true);
}

} // namespace sbx
