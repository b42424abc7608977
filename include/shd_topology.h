/*
 * shd_topology.h — drop-in replacement for Shadow's routing API.
 *
 * Every prototype below is signature-identical to the one it replaces in
 *   /root/reference/src/main/routing/shd-topology.h:12-22
 * so Shadow's callers (host_boot shd-host.c:277, host_shutdown shd-host.c:136,
 * the connect() check shd-host.c:1165, worker_sendPacket shd-worker.c:238,246,
 * master_getLatency shd-master.c:444, _master_loadTopology shd-master.c:209,
 * master_free shd-master.c:100) link against libshdtopology.so unchanged.
 *
 * The implementation lives in shadow_amd/csrc/topology.cpp.  Path computation
 * runs on MI355X through the thin device C-ABI declared in shdr.h.
 *
 * GLib scalar typedefs are declared locally (ABI-identical to glib's gchar,
 * gdouble, gboolean, guint64) because this image ships no GLib dev headers.
 * When built inside Shadow, define SHD_TOPOLOGY_HAVE_GLIB before including this
 * header to use glib's own typedefs.
 */
#ifndef SHD_TOPOLOGY_DROPIN_H_
#define SHD_TOPOLOGY_DROPIN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef SHD_TOPOLOGY_HAVE_GLIB
typedef char gchar;
typedef double gdouble;
typedef int gboolean;
typedef uint64_t guint64;
#endif

/* Opaque handles, as in Shadow (shd-topology.h:12, shd-address.h, shd-random.h). */
typedef struct _Topology Topology;
typedef struct _Address Address;
typedef struct _Random Random;

/* shd-topology.h:14 / shd-topology.c:1343-1365. Returns NULL on parse or
 * validation failure (not strongly connected, unreadable file). The file is
 * read eagerly: Shadow unlinks graphPath right after this returns
 * (shd-master.c:210). */
Topology* topology_new(const gchar* graphPath);

/* shd-topology.h:15 / shd-topology.c:1305-1341. */
void topology_free(Topology* top);

/* shd-topology.h:17-18 / shd-topology.c:1260-1294 (hint filtering and the
 * rand_r-driven uniform pick of _topology_findAttachmentVertex :1174-1258). */
void topology_attach(Topology* top, Address* address, Random* randomSourcePool,
        gchar* ipHint, gchar* geocodeHint, gchar* typeHint, guint64* bwDownOut, guint64* bwUpOut);

/* shd-topology.h:19 / shd-topology.c:1296-1303. */
void topology_detach(Topology* top, Address* address);

/* shd-topology.h:20 / shd-topology.c:1066-1069: getLatency > -1. */
gboolean topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress);

/* shd-topology.h:21 / shd-topology.c:1046-1054: path latency in ms, -1 on failure. */
gdouble topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress);

/* shd-topology.h:22 / shd-topology.c:1056-1064: product of (1-loss), -1 on failure. */
gdouble topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress);

/* ---- symbols the drop-in imports from Shadow (shd-address.h:67,75,91,93,
 * shd-random.c:37-41, shd-worker.h:42). libshdtopology.so carries WEAK
 * definitions of these for standalone use (shadow_amd/csrc/shim.c); Shadow's
 * strong definitions win when linked into the simulator. ---- */
uint32_t address_toNetworkIP(Address* address);
const gchar* address_toHostIPString(Address* address);
const gchar* address_toString(Address* address);
uint32_t address_stringToIP(const gchar* ipString);
gdouble random_nextDouble(Random* random);
void worker_updateMinTimeJump(gdouble minPathLatency);

/* ---- standalone-harness helpers (not part of Shadow's API; only defined by
 * the weak shim, used by tests/bench to build Address/Random objects). ---- */
Address* shdtop_address_new(uint32_t networkIP, const gchar* name);
void shdtop_address_free(Address* address);
Random* shdtop_random_new(unsigned int seed);
void shdtop_random_free(Random* random);
/* last value delivered through the (shim) worker_updateMinTimeJump upcall,
 * and how many upcalls were made. */
gdouble shdtop_last_min_time_jump(void);
uint64_t shdtop_min_time_jump_calls(void);
void shdtop_reset_min_time_jump(void);
/* the first (up to 4096) upcall values in call order: copies min(n, recorded)
 * of them to out and returns the number of upcalls made */
uint64_t shdtop_min_time_jump_history(gdouble* out, uint64_t n);

/* Introspection for tests and integration: number of path rows revealed so far,
 * whether the loaded graph took the complete-graph branch, and the running
 * minimum path latency (shd-topology.c:30,602-606). */
int topology_debug_isComplete(Topology* top);
int topology_debug_isDirected(Topology* top);
gdouble topology_debug_minimumPathLatency(Topology* top);
int32_t topology_debug_vertexOf(Topology* top, Address* address);
/* Phases of the last table computation (milliseconds unless noted): out[0]
 * engine creation (the call that created the engines, else 0), out[1] the last
 * row block's wall time, out[2] its rows (count), out[3..8] the first engine's
 * host phases of that block: landmark pre-pass, source grouping, launch,
 * pass (kernels), exposed device-to-host copy, total. Fills min(n, 9), returns 9. */
int topology_debug_lastComputeTimes(Topology* top, double* out, int n);
/* Row blocks of the current table: returns the block count (0 before the first
 * query), rows per block (the first block's) and how many are computed. */
int topology_debug_tableBlocks(Topology* top, int32_t* rowsPerBlockOut, int32_t* computedOut);

#ifdef __cplusplus
}
#endif

#endif /* SHD_TOPOLOGY_DROPIN_H_ */
