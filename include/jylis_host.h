/* jylis_host.h -- C ABI of the host mirror: Database / RepoManagerCore /
 * Repo* over the GPU engine (jylis_amd/csrc/host_repo.hip).
 *
 * This is the host side ABOVE the drop-in boundary (include/jylis_gpu.h),
 * written in C++ because the reference host is compiled Pony and ponyc is not
 * available here.  It mirrors the reference's operator interface for the
 * converge path and the commands around it:
 *   Database.apply            jylis/database.pony:25-40   -> jyh_db_apply
 *   Database.flush_deltas     jylis/database.pony:42-48   -> jyh_db_flush
 *   Database.converge_deltas  jylis/database.pony:50-51   -> jyh_db_converge
 *   Database.clean_shutdown   jylis/database.pony:53-65   -> jyh_db_shutdown
 * Replies are RESP bytes as jemc/pony-resp writes them (+OK, :n, $len, *n,
 * -ERR).  Delta batches travel as an engine-neutral byte blob (the Pony
 * runtime serialisation of _serialise.pony:9-14 is out of scope).
 */
#ifndef JYLIS_HOST_H
#define JYLIS_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct jyh_db jyh_db;

/* one node: identity = Address.hash64 (address.pony:29-33), one GPU */
int32_t jyh_db_create(int32_t device, uint64_t identity, jyh_db** out);
void jyh_db_destroy(jyh_db* db);
const char* jyh_db_error(const jyh_db* db);

/* one parsed RESP command (argv[0] = data type); the reply goes to out */
int32_t jyh_db_apply(jyh_db* db, uint32_t argc, const char* const* argv, const uint64_t* lens, uint8_t* out,
                     uint64_t cap, uint64_t* out_len);
/* flush every repo's pending deltas into one blob (malloc'd; jyh_free) */
int32_t jyh_db_flush(jyh_db* db, uint8_t** out, uint64_t* len);
/* converge a blob produced by a peer's jyh_db_flush */
int32_t jyh_db_converge(jyh_db* db, const uint8_t* blob, uint64_t len);
/* stop accepting commands (they answer SHUTDOWN), flush handled by caller */
int32_t jyh_db_shutdown(jyh_db* db);
void jyh_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* JYLIS_HOST_H */
