/* erl_nif.h DECLARATIONS ONLY, restated from the erl_nif API documentation, so that
 * c_src/deltagpu_nif.c can be syntax- and type-checked (gcc -fsyntax-only) in an image
 * without Erlang/OTP.  Not OTP's header and never linked: the NIF is built by the Elixir
 * project against its own OTP. */
#ifndef DG_ERL_NIF_DECLS_H
#define DG_ERL_NIF_DECLS_H
#include <stddef.h>
#include <stdint.h>

typedef unsigned long ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef struct ErlDrvMutex ErlNifMutex;
typedef long ErlNifSInt64;
typedef unsigned long ErlNifUInt64;
typedef struct {
  size_t size;
  unsigned char* data;
  void* ref_bin;
  void* __spare__[2];
} ErlNifBinary;
typedef struct {
  ERL_NIF_TERM map;
  size_t size, idx;
  void* u[4];
} ErlNifMapIterator;
typedef enum { ERL_NIF_MAP_ITERATOR_FIRST = 1, ERL_NIF_MAP_ITERATOR_LAST = 2 } ErlNifMapIteratorEntry;
typedef enum { ERL_NIF_LATIN1 = 1, ERL_NIF_UTF8 = 2 } ErlNifCharEncoding;
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef enum {
  ERL_NIF_TERM_TYPE_ATOM = 1, ERL_NIF_TERM_TYPE_BITSTRING = 2, ERL_NIF_TERM_TYPE_FLOAT = 3,
  ERL_NIF_TERM_TYPE_FUN = 4, ERL_NIF_TERM_TYPE_INTEGER = 5, ERL_NIF_TERM_TYPE_LIST = 6,
  ERL_NIF_TERM_TYPE_MAP = 7, ERL_NIF_TERM_TYPE_PID = 8, ERL_NIF_TERM_TYPE_PORT = 9,
  ERL_NIF_TERM_TYPE_REFERENCE = 10, ERL_NIF_TERM_TYPE_TUPLE = 11
} ErlNifTermType;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
typedef struct {
  const char* name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv*, int, const ERL_NIF_TERM[]);
  unsigned flags;
} ErlNifFunc;

int enif_compare(ERL_NIF_TERM, ERL_NIF_TERM);
int enif_is_identical(ERL_NIF_TERM, ERL_NIF_TERM);
int enif_is_empty_list(ErlNifEnv*, ERL_NIF_TERM);
ErlNifTermType enif_term_type(ErlNifEnv*, ERL_NIF_TERM);
int enif_get_int(ErlNifEnv*, ERL_NIF_TERM, int*);
int enif_get_uint(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_int64(ErlNifEnv*, ERL_NIF_TERM, ErlNifSInt64*);
int enif_get_uint64(ErlNifEnv*, ERL_NIF_TERM, ErlNifUInt64*);
int enif_get_double(ErlNifEnv*, ERL_NIF_TERM, double*);
int enif_get_tuple(ErlNifEnv*, ERL_NIF_TERM, int*, const ERL_NIF_TERM**);
int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_map_size(ErlNifEnv*, ERL_NIF_TERM, size_t*);
int enif_get_map_value(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM*);
int enif_get_atom_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*, ErlNifCharEncoding);
int enif_get_atom(ErlNifEnv*, ERL_NIF_TERM, char*, unsigned, ErlNifCharEncoding);
int enif_get_resource(ErlNifEnv*, ERL_NIF_TERM, ErlNifResourceType*, void**);
int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
int enif_term_to_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
int enif_alloc_binary(size_t, ErlNifBinary*);
void enif_release_binary(ErlNifBinary*);
int enif_map_iterator_create(ErlNifEnv*, ERL_NIF_TERM, ErlNifMapIterator*, ErlNifMapIteratorEntry);
int enif_map_iterator_get_pair(ErlNifEnv*, ErlNifMapIterator*, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_map_iterator_next(ErlNifEnv*, ErlNifMapIterator*);
void enif_map_iterator_destroy(ErlNifEnv*, ErlNifMapIterator*);
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char*);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv*);
ERL_NIF_TERM enif_make_binary(ErlNifEnv*, ErlNifBinary*);
unsigned char* enif_make_new_binary(ErlNifEnv*, size_t, ERL_NIF_TERM*);
ERL_NIF_TERM enif_make_copy(ErlNifEnv*, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_int(ErlNifEnv*, int);
ERL_NIF_TERM enif_make_int64(ErlNifEnv*, ErlNifSInt64);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv*, ErlNifUInt64);
ERL_NIF_TERM enif_make_list(ErlNifEnv*, unsigned, ...);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv*, const ERL_NIF_TERM*, unsigned);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_new_map(ErlNifEnv*);
int enif_make_map_put(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM*);
int enif_make_map_from_arrays(ErlNifEnv*, ERL_NIF_TERM[], ERL_NIF_TERM[], size_t, ERL_NIF_TERM*);
ERL_NIF_TERM enif_make_resource(ErlNifEnv*, void*);
ERL_NIF_TERM enif_make_string(ErlNifEnv*, const char*, ErlNifCharEncoding);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
void* enif_alloc(size_t);
void enif_free(void*);
ErlNifEnv* enif_alloc_env(void);
void enif_free_env(ErlNifEnv*);
void* enif_alloc_resource(ErlNifResourceType*, size_t);
void enif_release_resource(void*);
int enif_keep_resource(void*);
ErlNifResourceType* enif_open_resource_type(ErlNifEnv*, const char*, const char*, ErlNifResourceDtor*,
                                            ErlNifResourceFlags, ErlNifResourceFlags*);
ErlNifMutex* enif_mutex_create(char*);
void enif_mutex_destroy(ErlNifMutex*);
void enif_mutex_lock(ErlNifMutex*);
void enif_mutex_unlock(ErlNifMutex*);

#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD) \
  const ErlNifFunc* dg_nif_funcs = FUNCS;                        \
  int (*dg_nif_load)(ErlNifEnv*, void**, ERL_NIF_TERM) = LOAD;
#endif
