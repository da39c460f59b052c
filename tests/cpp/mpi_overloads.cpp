// Type-checks the MPI_Comm overloads of include/superbblas.h (compiled with -fsyntax-only
// against tests/cpp/mpi_stub; see tests/test_cpu_header.py).
#include "superbblas.h"

using namespace superbblas;
using Z = std::complex<double>;

void use_mpi_overloads(MPI_Comm comm) {
    Context gpu = createGpuContext(0);
    const Coor<2> d{4, 4};
    PartitionItem<2> p{Coor<2>{}, d};
    const Z *c0 = nullptr;
    Z *v1 = nullptr;
    copy<2, 2, Z, Z>(1.0, &p, 1, "ab", Coor<2>{}, d, d, &c0, nullptr, &gpu, &p, 1, "ba", Coor<2>{},
                     d, &v1, nullptr, &gpu, comm, SlowToFast, Copy);
    const PartitionItem<1> pr{Coor<1>{}, Coor<1>{4}};
    contraction<2, 2, 1, Z>(Z(1), &p, Coor<2>{}, d, d, 1, "ab", false, &c0, &gpu, &p, Coor<2>{},
                            d, d, 1, "ab", true, &c0, &gpu, Z(0), &pr, Coor<1>{}, Coor<1>{4},
                            Coor<1>{4}, 1, "a", &v1, &gpu, comm, SlowToFast);
    IndexType *ii = nullptr;
    Coor<2> *jj = nullptr;
    BSR_handle *op = nullptr;
    create_bsr<2, 2, Z>(&p, d, &p, d, 1, Coor<2>{1, 1}, Coor<2>{1, 1}, false, &ii, &jj, &c0, &gpu,
                        comm, SlowToFast, &op);
    create_kron_bsr<2, 2, Z>(&p, d, &p, d, 1, Coor<2>{1, 1}, Coor<2>{1, 1}, Coor<2>{1, 1},
                             Coor<2>{1, 1}, false, &ii, &jj, &c0, &c0, &gpu, comm, SlowToFast,
                             &op);
    cholesky<2, Z>(&p, d, 1, "ab", &v1, "a", "b", &gpu, comm, SlowToFast);
    inversion<2, Z>(&p, d, 1, "ab", &v1, "a", "b", &gpu, comm, SlowToFast);
    trsm<2, 2, 2, Z>(Z(1), &p, d, 1, "ab", &c0, "a", "b", &gpu, &p, d, 1, "bn", &c0, &gpu, &p, d,
                     1, "an", &v1, &gpu, comm, SlowToFast);
    gesm<2, 2, 2, Z>(Z(1), &p, d, 1, "ab", &c0, "a", "b", &gpu, &p, d, 1, "bn", &c0, &gpu, &p, d,
                     1, "an", &v1, &gpu, comm, SlowToFast);
    const PartitionItem<3> px{Coor<3>{}, Coor<3>{4, 4, 2}};
    bsr_krylov<2, 2, 3, 3, Z>(Z(1), op, "ab", "AB", &px, 1, "ABn", Coor<3>{}, Coor<3>{4, 4, 2},
                              Coor<3>{4, 4, 2}, &c0, Z(0), &px, "abn", Coor<3>{}, Coor<3>{4, 4, 2},
                              Coor<3>{4, 4, 2}, 0, &v1, &gpu, comm, SlowToFast);
    MatrixLayout lx, ly;
    bsr_get_preferred_layout<2, 2, Z>(op, 1, &gpu, comm, SlowToFast, &lx, &ly);
    Storage_handle sto = nullptr;
    create_storage<2, Z>(d, SlowToFast, "f", "", 0, NoChecksum, comm, &sto);
    open_storage<2, Z>("f", true, comm, &sto);
    append_blocks<2, Z>(&p, 1, d, sto, comm, SlowToFast);
    append_blocks<2, 2, Z>(&p, 1, "ab", Coor<2>{}, d, d, "ba", Coor<2>{}, sto, comm, SlowToFast);
    save<2, 2, Z, Z>(Z(1), &p, 1, "ab", Coor<2>{}, d, d, &c0, &gpu, "ab", Coor<2>{}, sto, comm,
                     SlowToFast);
    load<2, 2, Z, Z>(Z(1), sto, "ab", Coor<2>{}, d, &p, 1, "ab", Coor<2>{}, d, &v1, &gpu, comm,
                     SlowToFast, Copy);
    std::vector<PartitionItem<2>> blocks;
    get_blocks<2, 2, Z>(sto, "ab", "ab", Coor<2>{}, d, blocks, comm, SlowToFast);
    values_datatype vt;
    std::vector<char> md;
    std::vector<IndexType> dims;
    read_storage_header("f", SlowToFast, vt, md, dims, comm);
    check_storage<2, Z>(sto, comm);
    close_storage<2, Z>(sto, comm);
}

// support API of the reference that needs no communicator (platform.h:818-821,
// runtime_features.h:15-158)
static_assert(supported_type<Z>::value && supported_type<const float>::value &&
                  supported_type<int>::value && !supported_type<char>::value,
              "supported_type");
bool runtime_features() {
    getTrackingTime() = true;
    getTrackingMemory() = false;
    return getLogLevel() + getDebugLevel() >= 0 && getUseMPINonBlock() && getUseAlltoall() &&
           getUseMPIGpu() >= -1 && getMaxCacheGiBCpu() < 1e9 && getMaxCacheGiBGpu() < 1e9 &&
           !getTrackingTimeSync();
}
