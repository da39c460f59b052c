/* Declarations-only stand-in for <mpi.h>, used solely to type-check the SUPERBBLAS_USE_MPI
   section of include/superbblas.h with -fsyntax-only (MPI is not installed in this image).
   Nothing is linked or run against it. */
#ifndef SBX_TEST_MPI_STUB_H
#define SBX_TEST_MPI_STUB_H
typedef int MPI_Comm;
typedef int MPI_Datatype;
#define MPI_SUCCESS 0
#define MPI_IDENT 0
#define MPI_UNEQUAL 3
#define MPI_BYTE ((MPI_Datatype)1)
#define MPI_COMM_WORLD ((MPI_Comm)0)
int MPI_Comm_size(MPI_Comm, int *);
int MPI_Comm_rank(MPI_Comm, int *);
int MPI_Comm_compare(MPI_Comm, MPI_Comm, int *);
typedef int MPI_Info;
#define MPI_INT ((MPI_Datatype)2)
#define MPI_INFO_NULL ((MPI_Info)0)
#define MPI_COMM_TYPE_SHARED 1
int MPI_Comm_split_type(MPI_Comm, int, int, MPI_Info, MPI_Comm *);
int MPI_Comm_free(MPI_Comm *);
int MPI_Allgather(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPI_Comm);
int MPI_Bcast(void *, int, MPI_Datatype, int, MPI_Comm);
int MPI_Alltoallv(const void *, const int *, const int *, MPI_Datatype, void *, const int *,
                  const int *, MPI_Datatype, MPI_Comm);
#endif
