/* fd_verify_gpu_tile.c -- the GPU tile of the service-mode verify stage, for
   the reference's topology.  It goes in the reference tree as
   src/disco/verify/fd_verify_gpu_tile.c (config/extra/with-hip.mk adds it to
   the build with FD_HAS_HIP_SVC; integration/fd_verify_topo_hip.patch adds
   the tiles, the verify_svc objects and the registrations).

   One "vgpu" tile per GPU (kind_id = the HIP device).  It owns the GPU's
   HIP context -- the only multithreaded tile, so the only one
   fd_sandbox_enter cannot take (its unshare( CLONE_NEWUSER ) refuses a
   threaded process, src/util/sandbox/fd_sandbox.c:649; the topology patch
   skips that call for it) -- and enters everything of the sandbox a
   threaded process can take in unprivileged_init
   (fd_hip_tile_sandbox_process, include/fd_hip_tile_sandbox.h): the fd
   allow-list, rlimits, no capabilities, no_new_privs and a seccomp filter
   over every thread of the process (SECCOMP_FILTER_FLAG_TSYNC).  It serves the verify
   tiles with kind_id % gpu_cnt == kind_id through its verify_svc object
   (include/fd_verify_svc.h): every quic_verify link's mcache and dcache and
   its tiles' verify_dedup dcaches are registered for the GPU in
   privileged_init, then the stem loop calls fd_verify_svc_poll from
   after_credit.  The verify tiles stay the reference's single-threaded,
   sandboxed processes (integration/fd_verify_tile_svc.patch).

   The same steps, on a run's shared file instead of the topology's
   workspaces, are integration/svc_run.c (what the tests and the bench run).

   Properties (topo->props, set by the topology patch):
     verify_svc.gpu_cnt            GPU tiles (verify tile kind_id % gpu_cnt picks one)
     verify_svc.<g>                obj id of GPU g's segment
     obj.<id>.{tile_cnt,req_depth,slot_cap,frag_cap}   the segment's shape
     verify_svc.batch_max, verify_svc.inflight         launch size and count
     verify_svc.merge_min, .merge_wait_ns, .merge_idle_ns   the merge policy (fd_verify_svc_set_merge)
     verify_svc.hw_queues          GPU_MAX_HW_QUEUES for this process (1..32)
   Defaults: the measured best on one MI355X, the
   same as integration/svc_run.c's. */

#define SVC_BATCH_MAX_DEFAULT     (262144UL)
#define SVC_INFLIGHT_DEFAULT      (2UL)
#define SVC_MERGE_WAIT_NS_DEFAULT (2000000UL)
#define SVC_MERGE_IDLE_NS_DEFAULT (20000UL)
#define SVC_HW_QUEUES_DEFAULT     (8UL)

#include <stdio.h>                            /* snprintf */
#include <stdlib.h>                           /* setenv */
#include "../topo/fd_topo.h"
#include "../../util/pod/fd_pod_format.h"
#include "../../tango/mcache/fd_mcache.h"
#include "../../tango/dcache/fd_dcache.h"
#include "fd_verify_svc.h"
#include "fd_hip_tile_sandbox.h"

#define VAL(name) (__extension__({                                                             \
  ulong __x = fd_pod_queryf_ulong( topo->props, ULONG_MAX, "obj.%lu.%s", obj->id, name );      \
  if( FD_UNLIKELY( __x==ULONG_MAX ) ) FD_LOG_ERR(( "obj.%lu.%s was not set", obj->id, name )); \
  __x; }))

/* ---- the verify_svc object (fd_topo_obj_callbacks_t, as src/app/shared/fd_obj_callbacks.c) ---- */

static ulong
verify_svc_footprint( fd_topo_t const * topo, fd_topo_obj_t const * obj ) {
  ulong fp = fd_verify_svc_footprint( VAL("tile_cnt"), VAL("req_depth"), VAL("slot_cap"), VAL("frag_cap") );
  if( FD_UNLIKELY( !fp ) ) FD_LOG_ERR(( "obj.%lu: bad verify_svc shape", obj->id ));
  return fp;
}

static ulong
verify_svc_align( fd_topo_t const * topo FD_FN_UNUSED, fd_topo_obj_t const * obj FD_FN_UNUSED ) {
  return FD_VERIFY_SVC_ALIGN;
}

static void
verify_svc_new( fd_topo_t const * topo, fd_topo_obj_t const * obj ) {
  FD_TEST( fd_verify_svc_new( fd_topo_obj_laddr( topo, obj->id ), VAL("tile_cnt"), VAL("req_depth"), VAL("slot_cap"),
                              VAL("frag_cap") ) );
}

fd_topo_obj_callbacks_t fd_obj_cb_verify_svc = {
  .name      = "verify_svc",
  .footprint = verify_svc_footprint,
  .align     = verify_svc_align,
  .new       = verify_svc_new,
};

/* ---- the tile ---------------------------------------------------------------------------- */

typedef struct {
  fd_verify_svc_t * svc;
  ulong             mapped[ FD_TOPO_MAX_WKSPS ];   /* workspaces registered for the GPU */
} fd_vgpu_ctx_t;

FD_FN_CONST static inline ulong scratch_align( void ) { return 128UL; }
FD_FN_PURE  static inline ulong scratch_footprint( fd_topo_tile_t const * tile ) { (void)tile; return sizeof(fd_vgpu_ctx_t); }

/* register a workspace for the GPU once (all of it: links' mcaches,
   dcaches and the segment are addressed inside it) */
static void
vgpu_map( fd_vgpu_ctx_t * ctx, fd_topo_t const * topo, ulong wksp_id ) {
  if( ctx->mapped[ wksp_id ] ) return;
  fd_topo_wksp_t const * w = &topo->workspaces[ wksp_id ];
  if( FD_UNLIKELY( fd_verify_svc_map( ctx->svc, w->wksp, w->page_sz*w->page_cnt ) ) )
    FD_LOG_ERR(( "registering workspace %s (%lu B) for the GPU failed", w->name, w->page_sz*w->page_cnt ));
  ctx->mapped[ wksp_id ] = 1UL;
}

static void
privileged_init( fd_topo_t * topo, fd_topo_tile_t * tile ) {
  fd_vgpu_ctx_t * ctx = (fd_vgpu_ctx_t *)fd_topo_obj_laddr( topo, tile->tile_obj_id );
  memset( ctx, 0, sizeof(fd_vgpu_ctx_t) );
  ulong gpu     = tile->kind_id;
  ulong gpu_cnt = fd_pod_query_ulong( topo->props, "verify_svc.gpu_cnt", 0UL );
  ulong obj_id  = fd_pod_queryf_ulong( topo->props, ULONG_MAX, "verify_svc.%lu", gpu );
  if( FD_UNLIKELY( !gpu_cnt || gpu>=gpu_cnt || obj_id==ULONG_MAX ) ) FD_LOG_ERR(( "no verify_svc object for GPU %lu", gpu ));
  /* before the first HIP call: hardware queues for the ingest, flush and
     launch streams (HIP's default 4 makes the ingest and flush streams wait
     behind verify launches in shared queues); set
     over the environment's value, which is HIP's default on hosts that
     export it (verify_svc.hw_queues, default 8) */
  {
    ulong hwq = fd_pod_query_ulong( topo->props, "verify_svc.hw_queues", SVC_HW_QUEUES_DEFAULT );
    if( FD_UNLIKELY( hwq<1UL || hwq>32UL ) ) FD_LOG_ERR(( "verify_svc.hw_queues %lu not in [1,32]", hwq ));
    char q[ 24 ];
    snprintf( q, sizeof(q), "%lu", hwq );
    setenv( "GPU_MAX_HW_QUEUES", q, 1 );
  }
  ulong batch_max = fd_pod_query_ulong( topo->props, "verify_svc.batch_max", SVC_BATCH_MAX_DEFAULT );
  ulong inflight  = fd_pod_query_ulong( topo->props, "verify_svc.inflight",  SVC_INFLIGHT_DEFAULT  );
  ctx->svc = fd_verify_svc_boot( fd_topo_obj_laddr( topo, obj_id ), (int)gpu, batch_max, inflight );
  if( FD_UNLIKELY( !ctx->svc ) ) FD_LOG_ERR(( "fd_verify_svc_boot failed on GPU %lu", gpu ));
  fd_verify_svc_set_merge( ctx->svc, fd_pod_query_ulong( topo->props, "verify_svc.merge_min", batch_max/2UL ),
                           fd_pod_query_ulong( topo->props, "verify_svc.merge_wait_ns", SVC_MERGE_WAIT_NS_DEFAULT ),
                           fd_pod_query_ulong( topo->props, "verify_svc.merge_idle_ns", SVC_MERGE_IDLE_NS_DEFAULT ) );
  vgpu_map( ctx, topo, topo->objs[ obj_id ].wksp_id );

  /* every quic_verify link (service link l = its kind_id) */
  for( ulong i=0UL; i<topo->link_cnt; i++ ) {
    fd_topo_link_t const * l = &topo->links[ i ];
    if( strcmp( l->name, "quic_verify" ) ) continue;
    ulong dw = topo->objs[ l->dcache_obj_id ].wksp_id;
    vgpu_map( ctx, topo, topo->objs[ l->mcache_obj_id ].wksp_id );
    vgpu_map( ctx, topo, dw );
    void * base = topo->workspaces[ dw ].wksp;
    if( FD_UNLIKELY( fd_verify_svc_set_link( ctx->svc, l->kind_id, l->mcache, fd_mcache_depth( l->mcache ), base,
                                             fd_dcache_compact_chunk0( base, l->dcache ),
                                             fd_dcache_compact_wmark ( base, l->dcache, l->mtu ) ) ) )
      FD_LOG_ERR(( "quic_verify link %lu: fd_verify_svc_set_link failed", l->kind_id ));
  }
  /* the verify tiles this GPU serves: their verify_dedup dcaches */
  for( ulong i=0UL; i<topo->tile_cnt; i++ ) {
    fd_topo_tile_t const * v = &topo->tiles[ i ];
    if( strcmp( v->name, "verify" ) || fd_verify_svc_gpu_of( v->kind_id, gpu_cnt )!=gpu ) continue;
    fd_topo_link_t const * out = &topo->links[ v->out_link_id[ 0 ] ];
    ulong dw = topo->objs[ out->dcache_obj_id ].wksp_id;
    vgpu_map( ctx, topo, dw );
    if( FD_UNLIKELY( fd_verify_svc_set_tile( ctx->svc, fd_verify_svc_slot_of( v->kind_id, gpu_cnt ), out->dcache,
                                             fd_dcache_data_sz( out->dcache ), topo->workspaces[ dw ].wksp ) ) )
      FD_LOG_ERR(( "verify tile %lu: fd_verify_svc_set_tile failed", v->kind_id ));
  }
  /* GPU 0's clients (the shred tiles' FEC-set roots, the replay tile's
     block sigverify; include/fd_verify_svc.h "clients"): segment tiles
     [verify_svc.client_base, +verify_svc.client_cnt), after its verify tiles */
  if( gpu==0UL ) {
    ulong cb = fd_pod_query_ulong( topo->props, "verify_svc.client_base", 0UL );
    ulong cc = fd_pod_query_ulong( topo->props, "verify_svc.client_cnt",  0UL );
    for( ulong c=0UL; c<cc; c++ )
      if( FD_UNLIKELY( fd_verify_svc_set_client( ctx->svc, cb+c ) ) ) FD_LOG_ERR(( "client tile %lu: fd_verify_svc_set_client failed", cb+c ));
  }
  if( FD_UNLIKELY( fd_verify_svc_run( ctx->svc ) ) ) FD_LOG_ERR(( "fd_verify_svc_run failed (a verify tile not set?)" ));
}

/* after fd_topo_run_tile's uid / gid switch: the sandbox of a threaded
   process (the HIP runtime's threads included), every HIP resource already
   set up in privileged_init.  A call outside the filter kills the process,
   as fd_sandbox's SECCOMP_RET_KILL_PROCESS policies do. */
static void
unprivileged_init( fd_topo_t * topo, fd_topo_tile_t * tile ) {
  (void)topo; (void)tile;
  int  dev[ FD_HIP_TILE_FD_MAX ];
  long nd = fd_hip_tile_device_fds( dev, FD_HIP_TILE_FD_MAX );
  if( FD_UNLIKELY( nd<0L ) ) FD_LOG_ERR(( "the HIP device fds could not be listed" ));
  char why[ 160 ];
  if( FD_UNLIKELY( fd_hip_tile_sandbox_process( fd_log_private_logfile_fd(), dev, (ulong)nd, 0, SECCOMP_RET_KILL_PROCESS,
                                                why, sizeof(why) ) ) )
    FD_LOG_ERR(( "vgpu sandbox: %s", why ));
}

static inline void
after_credit( fd_vgpu_ctx_t *     ctx,
              fd_stem_context_t * stem,
              int *               opt_poll_in,
              int *               charge_busy ) {
  (void)stem; (void)opt_poll_in;
  *charge_busy = fd_verify_svc_poll( ctx->svc );
}

#define STEM_BURST                  (1UL)
#define STEM_CALLBACK_CONTEXT_TYPE  fd_vgpu_ctx_t
#define STEM_CALLBACK_CONTEXT_ALIGN 128UL
#define STEM_CALLBACK_AFTER_CREDIT  after_credit

#include "../stem/fd_stem.c"

fd_topo_run_tile_t fd_tile_verify_gpu = {
  .name                     = "vgpu",
  .scratch_align            = scratch_align,
  .scratch_footprint        = scratch_footprint,
  .privileged_init          = privileged_init,
  .unprivileged_init        = unprivileged_init,
  .run                      = stem_run,
};
