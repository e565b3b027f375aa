/* svc_run.h -- the shared-memory layout of the service-mode verify stage
   run (integration/svc_tile_run.c: producer, verify tiles, consumers;
   integration/svc_run.c: the GPU tile).  One file in /dev/shm holds every
   link of the stage, as the reference's workspaces would:

     run header                      svc_run_hdr_t
     per quic_verify link l          mcache (in_depth), the tiles' fseqs, dcache
     per verify tile t               verify_dedup mcache (out_depth) and dcache
                                     (fd_dcache_req_data_sz( FD_TPU_PARSED_MTU,
                                     out_depth, 1, 1 ): the reference's sizing,
                                     burst 1), its consumer's fseq
     the verify service segment      fd_verify_svc_new( ... )

   Offsets are page-aligned (the GPU tile registers the whole file once).
   Chunks of every link are relative to the file's base, which stands in
   for each link's workspace. */
#ifndef HEADER_svc_run_h
#define HEADER_svc_run_h

#define SVC_RUN_MAGIC     (0xfd75c7a11e5a11ceUL)
#define SVC_RUN_TILE_MAX  (16UL)
#define SVC_RUN_LINK_MAX  (4UL)
#define SVC_RUN_LAT_B     (128UL)       /* latency histogram: bucket k covers [2^(k/4), 2^((k+1)/4)) ns */

typedef struct {
  volatile long  t_end;
  volatile ulong done, frags, sigs, pub, parse, verify, dedup, bundle, overrun, lapped, host, early;
  volatile ulong regime[ 8 ];                  /* the stem's REGIME_DURATION_NANOS ticks (fd_stem.c:406-712) */
  volatile ulong link_consumed, link_filtered, link_ovr_poll, link_ovr_poll_frags, link_ovr_read, link_ovr_read_frags;
  volatile ulong metrics_ok;                   /* the link-in metric slots hold the tile's counts */
  volatile ulong threads, dev_fds;             /* after privileged_init: /proc/self/task entries, /dev/kfd|dri fds */
  volatile ulong sandboxed;                    /* the tile ran inside fd_sandbox_enter (SVC_RUN_SANDBOX) */
  volatile double sec_pub, sec_pass, sec_flush, sec_post;   /* the tile's time in before_credit's steps */
  volatile ulong m_sigs, m_host;               /* the VERIFY_GPU_SIGNATURES / _HOST_REDONE metric slots */
  volatile ulong m_ing_n, m_ing_sum, m_batch_n, m_batch_sum;   /* the two GPU latency histograms' samples and sums (ns) */
  volatile ulong ing_p50, ing_p99, ing_max;    /* post -> INGESTED as the tile saw it (ns; bucket right edges; max: the
                                                  highest nonempty bucket's) */
} svc_run_tile_res_t;

typedef struct {
  volatile ulong done, frags, bytes, digest, overrun, bad;
  volatile long  t_last;                       /* wallclock of the last frag */
  volatile ulong lat[ SVC_RUN_LAT_B ];         /* tspub - tsorig, ns */
  volatile ulong lat_q[ SVC_RUN_LAT_B ];       /* now - tsorig at consume, ns */
} svc_run_cons_res_t;

typedef struct {
  ulong magic;
  ulong n, tile_cnt, seed, tcache_depth, in_depth, link_cnt, out_depth;
  ulong mcache_off[ SVC_RUN_LINK_MAX ], dcache_off[ SVC_RUN_LINK_MAX ], fseq_off[ SVC_RUN_LINK_MAX ];
  ulong fseq_stride, dcache_data_sz;
  ulong out_mcache_off[ SVC_RUN_TILE_MAX ], out_dcache_off[ SVC_RUN_TILE_MAX ], cons_fseq_off[ SVC_RUN_TILE_MAX ];
  ulong out_data_sz;
  ulong svc_off, svc_sz, req_depth, slot_cap, frag_cap;
  ulong client_cnt;                            /* the segment's last client_cnt tiles are clients (FD_VERIFY_SVC_REQ_SIGS:
                                                  integration/svc_client.h), after the tile_cnt verify tiles */
  volatile ulong clients_ready, clients_done;
  ulong map_sz;
  volatile ulong tiles_ready, cons_ready, svc_ready, start, shutdown, svc_done;
  volatile long  t0, t_pub;
  volatile ulong svc_stats[ 16 ];
  volatile ulong svc_occ[ 6 ];                 /* fd_verify_svc_occupancy */
  volatile ulong svc_pid;                      /* the GPU tile's process (its /proc task census, svc_tile_run produce) */
  volatile ulong svc_sandboxed;                /* the GPU tile entered fd_hip_tile_sandbox_process */
  volatile ulong svc_traps, svc_trap_nr[ 16 ]; /* SVC_SANDBOX=trap: syscalls the filter refused (their numbers) */
  svc_run_tile_res_t tile[ SVC_RUN_TILE_MAX ];
  svc_run_cons_res_t cons[ SVC_RUN_TILE_MAX ];
} svc_run_hdr_t;

#endif /* HEADER_svc_run_h */
