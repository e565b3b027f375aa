/* sched_run.c -- TEST INFRASTRUCTURE: one block through the reference's
   replay scheduler (src/discof/replay/fd_sched.c with
   integration/fd_replay_hip.patch), its sigverify retired in one of three
   ways:

     exec   the reference's own path: FD_SCHED_TT_TXN_SIGVERIFY tasks on
            emulated exec tiles, each running fd_executor_txn_verify
            (fd_executor.c:1607-1623: fd_ed25519_verify_batch_single_msg,
            the reference's CPU code, linked from its sources)
     claim  the patch's bulk path (fd_sched_sigverify_claim / _claim_done),
            each claimed batch verified by the same reference CPU function:
            checks the scheduler half of the patch without a GPU
     skip   the bulk path with every claimed transaction passed unverified:
            the scheduler and driver loop alone (the cost the other modes
            add to the replay thread is theirs minus this)
     hip    the patch's bulk path as the replay tile runs it
            (replay_hip_sigverify in fd_replay_tile.c): claimed batches
            packed into pinned buffers and verified by
            fd_replay_hip_txn_verify_host on the GPU, polled without blocking
     svc    the bulk path as the replay tile runs it in service mode
            (FD_HAS_HIP_SVC, _build/sched_run_svc): claimed batches become
            the GPU tile's signature records (include/fd_replay_svc.h) --
            no HIP in this process; a client of the run named by
            SVC_CLIENT_SHM (integration/svc_client.h)

   Exec tiles are emulated: a dispatched task completes one loop iteration
   later (tasks on several tiles overlap).  Banks are emulated by a refcnt
   and a dead flag per bank index.  As in the replay tile, a failed
   sigverify marks the bank dead and abandons the block (fd_sched_block_
   abandon) unless the run is in record mode, which keeps verifying so that
   every transaction's result can be compared.

   usage: sched_run <fecs.bin> <exec|claim|skip|hip|svc> <exec_cnt> <record 0|1> <out.bin> [batch_max] [batch_min]
   fecs.bin : "FDB1" u64 fec_cnt, then per FEC set: u32 data_sz, u8 last_in_batch, data
              (one block, bank 1 on the snapshot root bank 0; the last FEC
              set is the block's last)
   out.bin  : "FDR1" u64 cnt, then per sigverify: sig0[64] i32 result u8 source(1 exec, 2 bulk) u8[3]
   stdout   : one JSON line (counts, block state, seconds) */

#include "fd_sched.h"
#include "../../ballet/ed25519/fd_ed25519.h"
#include "../../ballet/sha512/fd_sha512.h"
#include "../../flamenco/runtime/fd_runtime_err.h"
#if FD_HAS_HIP
#include "fd_replay_hip.h"
#endif
#if FD_HAS_HIP_SVC
#include "fd_replay_svc.h"
#include "svc_client.h"
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#if defined(fd_boot)
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

#define BANK_CNT  (4UL)
#define EXEC_MAX  (64UL)
#define MODE_EXEC  0
#define MODE_CLAIM 1
#define MODE_HIP   2
#define MODE_SKIP  3
#define MODE_SVC   4

typedef struct { uchar sig0[ 64 ]; int result; uchar source; uchar pad[ 3 ]; } rec_t;
FD_STATIC_ASSERT( sizeof(rec_t)==72UL, rec_layout );

static rec_t * recs;
static ulong   rec_cnt, rec_max;
static ulong   bank_refcnt[ BANK_CNT ];
static int     bank_dead  [ BANK_CNT ];
static int     record_mode;
static ulong   sigs_exec, sigs_bulk, batches_bulk, bulk_max;
static double  t_ingest, t_bulk, t_sv_last, t_start;   /* ingest calls, bulk_sigverify calls, last sigverify done */
static fd_sha512_t * shas[ FD_TXN_ACTUAL_SIG_MAX ];

static double now( void ) { struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t ); return (double)t.tv_sec + 1e-9*(double)t.tv_nsec; }

/* fd_executor_txn_verify (fd_executor.c:1607-1623), the reference's code */
static int
txn_verify_ref( fd_txn_p_t * txn_p ) {
  fd_txn_t * txn = TXN( txn_p );
  int res = fd_ed25519_verify_batch_single_msg( txn_p->payload + txn->message_off,
                                                txn_p->payload_sz - txn->message_off,
                                                txn_p->payload + txn->signature_off,
                                                txn_p->payload + txn->acct_addr_off,
                                                shas, txn->signature_cnt );
  return res==FD_ED25519_SUCCESS ? FD_RUNTIME_EXECUTE_SUCCESS : FD_RUNTIME_TXN_ERR_SIGNATURE_FAILURE;
}

static void
record( fd_sched_t * sched, ulong txn_idx, int result, uchar source ) {
  FD_TEST( rec_cnt<rec_max );
  fd_txn_p_t * txn_p = fd_sched_get_txn( sched, txn_idx );
  rec_t * r = recs + rec_cnt++;
  memset( r, 0, sizeof(*r) );
  if( TXN( txn_p )->signature_cnt ) memcpy( r->sig0, txn_p->payload + TXN( txn_p )->signature_off, 64UL );
  r->result = result;
  r->source = source;
}

/* process_exec_task_done's failure handling (fd_replay_tile.c), banks
   emulated */
static void
sigverify_failed( fd_sched_t * sched, ulong bank_idx, int result ) {
  if( FD_UNLIKELY( result && !bank_dead[ bank_idx ] && !record_mode ) ) {
    bank_dead[ bank_idx ] = 1;
    fd_sched_block_abandon( sched, bank_idx );
  }
}

/* ---- bulk path: replay_hip_sigverify of the patch ------------------------ */

typedef struct {
  ulong   cnt, bank_idx;
  ulong * txn_idx;
  int *   result;
#if FD_HAS_HIP
  fd_replay_hip_t *   replay;
  uchar *             pool;
  fd_txn_hip_desc_t * desc;
#endif
#if FD_HAS_HIP_SVC
  fd_replay_svc_t *     svc;
  fd_replay_svc_txn_t * stx;
#endif
} bulk_t;

static int
bulk_sigverify( fd_sched_t * sched, bulk_t * b, int mode, ulong batch_min, ulong batch_max ) {
  if( b->cnt ) {
#if FD_HAS_HIP
    if( mode==MODE_HIP ) {
      int done = fd_replay_hip_poll( b->replay );
      if( !done ) return 0;
      FD_TEST( done==1 );
    }
#endif
#if FD_HAS_HIP_SVC
    if( mode==MODE_SVC && !fd_replay_svc_step( b->svc, fd_tickcount() ) ) return 0;
#endif
    for( ulong j=0UL; j<b->cnt; j++ ) {
      bank_refcnt[ b->bank_idx ]--;
      record( sched, b->txn_idx[ j ], b->result[ j ], 2 );
      sigverify_failed( sched, b->bank_idx, b->result[ j ] );
      fd_sched_sigverify_claim_done( sched, b->bank_idx, b->txn_idx[ j ] );
    }
    b->cnt = 0UL;
    t_sv_last = now() - t_start;
    return 1;
  }
  ulong bank_idx;
  ulong cnt = fd_sched_sigverify_claim( sched, batch_min, batch_max, &bank_idx, b->txn_idx );
  if( !cnt ) return 0;
  FD_TEST( bank_idx<BANK_CNT );
  bank_refcnt[ bank_idx ] += cnt;
  ulong sigs = 0UL;
  for( ulong j=0UL; j<cnt; j++ ) sigs += TXN( fd_sched_get_txn( sched, b->txn_idx[ j ] ) )->signature_cnt;
  sigs_bulk += sigs; batches_bulk++; bulk_max = fd_ulong_max( bulk_max, cnt );
  if( mode==MODE_CLAIM ) {
    for( ulong j=0UL; j<cnt; j++ ) b->result[ j ] = txn_verify_ref( fd_sched_get_txn( sched, b->txn_idx[ j ] ) );
  } else if( mode==MODE_SKIP ) {
    for( ulong j=0UL; j<cnt; j++ ) b->result[ j ] = FD_RUNTIME_EXECUTE_SUCCESS;
  } else {
#if FD_HAS_HIP
    ulong pool_sz = 0UL;
    for( ulong j=0UL; j<cnt; j++ ) {
      fd_txn_p_t const * txn_p = fd_sched_get_txn( sched, b->txn_idx[ j ] );
      fd_txn_t const *   txn   = TXN( txn_p );
      fd_memcpy( b->pool+pool_sz, txn_p->payload, txn_p->payload_sz );
      b->desc[ j ] = (fd_txn_hip_desc_t){ .payload_off   = (uint)pool_sz,
                                          .payload_sz    = (ushort)txn_p->payload_sz,
                                          .signature_off = txn->signature_off,
                                          .message_off   = txn->message_off,
                                          .acct_addr_off = txn->acct_addr_off,
                                          .signature_cnt = txn->signature_cnt };
      pool_sz += txn_p->payload_sz;
    }
    FD_TEST( !fd_replay_hip_txn_verify_host( b->replay, cnt, b->pool, pool_sz, b->desc, b->result, NULL ) );
#elif FD_HAS_HIP_SVC
    for( ulong j=0UL; j<cnt; j++ ) {
      fd_txn_p_t const * txn_p = fd_sched_get_txn( sched, b->txn_idx[ j ] );
      fd_txn_t const *   txn   = TXN( txn_p );
      b->stx[ j ] = (fd_replay_svc_txn_t){ .payload       = txn_p->payload,
                                           .payload_sz    = (ushort)txn_p->payload_sz,
                                           .signature_off = txn->signature_off,
                                           .message_off   = txn->message_off,
                                           .acct_addr_off = txn->acct_addr_off,
                                           .signature_cnt = txn->signature_cnt };
    }
    fd_replay_svc_start( b->svc, cnt, b->stx, b->result );
    (void)fd_replay_svc_step( b->svc, fd_tickcount() );
#else
    FD_LOG_ERR(( "hip / svc mode needs a FD_HAS_HIP / FD_HAS_HIP_SVC build" ));
#endif
  }
  b->cnt = cnt;
  b->bank_idx = bank_idx;
  return 1;
}

/* the scheduler's memory: fd_rdisp_new writes its whole account pool
   (depth FD_SCHED_MAX_DEPTH, ~28 GiB), so one region serves every job of
   a run, on transparent huge pages */
static void * sched_mem;

static int
run_job( char ** argv, int argc ) {
  if( argc<5 ) { fprintf( stderr, "job: fecs.bin exec|claim|skip|hip|svc exec_cnt record out.bin [batch_max] [batch_min]\n" ); return 2; }
  int mode = !strcmp( argv[1], "exec" ) ? MODE_EXEC : !strcmp( argv[1], "claim" ) ? MODE_CLAIM :
             !strcmp( argv[1], "hip" ) ? MODE_HIP : !strcmp( argv[1], "skip" ) ? MODE_SKIP :
             !strcmp( argv[1], "svc" ) ? MODE_SVC : -1;
  FD_TEST( mode>=0 );
  ulong exec_cnt  = strtoul( argv[2], NULL, 0 );
  record_mode     = atoi( argv[3] );
  ulong batch_max = argc>5 ? strtoul( argv[5], NULL, 0 ) : 16384UL;
  ulong batch_min = argc>6 ? strtoul( argv[6], NULL, 0 ) : 256UL;
  FD_TEST( exec_cnt>=1UL && exec_cnt<=EXEC_MAX && batch_max>=1UL );
  rec_cnt = 0UL; sigs_exec = sigs_bulk = batches_bulk = bulk_max = 0UL;
  memset( bank_refcnt, 0, sizeof(bank_refcnt) ); memset( bank_dead, 0, sizeof(bank_dead) );

  /* the block's FEC sets */
  FILE * f = fopen( argv[0], "rb" ); FD_TEST( f );
  char magic[ 4 ]; ulong fec_cnt;
  FD_TEST( fread( magic, 1, 4, f )==4 && !memcmp( magic, "FDB1", 4 ) && fread( &fec_cnt, 8, 1, f )==1 );
  fd_store_fec_t * fecs = aligned_alloc( alignof(fd_store_fec_t), fd_ulong_align_up( fec_cnt*sizeof(fd_store_fec_t), alignof(fd_store_fec_t) ) );
  uchar * last_in_batch = malloc( fec_cnt );
  FD_TEST( fecs && last_in_batch );
  ulong data_tot = 0UL;
  for( ulong i=0UL; i<fec_cnt; i++ ) {
    uint sz; uchar lb;
    FD_TEST( fread( &sz, 4, 1, f )==1 && fread( &lb, 1, 1, f )==1 && sz<=FD_STORE_DATA_MAX );
    memset( &fecs[ i ], 0, offsetof( fd_store_fec_t, data ) );
    FD_TEST( fread( fecs[ i ].data, 1, sz, f )==sz );
    fecs[ i ].data_sz = sz;
    for( ulong k=0UL; k<32UL; k++ ) fecs[ i ].block_offs[ k ] = (uint)( (ulong)sz*(k+1UL)/32UL );   /* 32 data shreds */
    last_in_batch[ i ] = lb;
    data_tot += sz;
  }
  fclose( f );

  fd_sched_t * sched = fd_sched_join( fd_sched_new( sched_mem, BANK_CNT, exec_cnt ), BANK_CNT );
  FD_TEST( sched );
  fd_sched_block_add_done( sched, 0UL, ULONG_MAX, 0UL );        /* the snapshot slot */

  rec_max = data_tot/FD_TXN_MIN_SERIALIZED_SZ + 1UL;
  recs    = malloc( rec_max*sizeof(rec_t) );
  FD_TEST( recs );

  bulk_t bulk[ 1 ] = {{ 0 }};
  bulk->txn_idx = malloc( batch_max*sizeof(ulong) );
  bulk->result  = malloc( batch_max*sizeof(int) );
  FD_TEST( bulk->txn_idx && bulk->result );
#if FD_HAS_HIP
  fd_ed25519_hip_ctx_t * hip = NULL;
  if( mode==MODE_HIP ) {
    hip = fd_ed25519_hip_ctx_new( 0, 16UL*batch_max );
    FD_TEST( hip );
    bulk->replay = fd_replay_hip_new( hip, batch_max );
    bulk->pool   = fd_ed25519_hip_host_alloc( FD_REPLAY_HIP_TXN_MTU*batch_max );
    bulk->desc   = fd_ed25519_hip_host_alloc( sizeof(fd_txn_hip_desc_t)*batch_max );
    int * res    = fd_ed25519_hip_host_alloc( sizeof(int)*batch_max );
    FD_TEST( bulk->replay && bulk->pool && bulk->desc && res );
    free( bulk->result );
    bulk->result = res;
  }
#endif
#if FD_HAS_HIP_SVC
  if( mode==MODE_SVC ) {
    /* one client per process: its request ring continues across jobs */
    static fd_replay_svc_t svc[1]; static int joined;
    if( !joined ) {
      ulong seg_t;
      fd_verify_svc_seg_t * seg = svc_client_attach( &seg_t );
      FD_TEST( fd_replay_svc_join( svc, seg, seg_t ) );
      joined = 1;
    }
    bulk->svc = svc;
    bulk->stx = malloc( batch_max*sizeof(fd_replay_svc_txn_t) );
    FD_TEST( bulk->stx );
  }
#endif

  struct { ulong type, txn_idx; } pend[ EXEC_MAX ];
  for( ulong k=0UL; k<EXEC_MAX; k++ ) pend[ k ].type = FD_SCHED_TT_NULL;
  ulong pend_cnt = 0UL, rr = 0UL, fec_i = 0UL, idle = 0UL;
  ulong tasks_exec = 0UL, tasks_sigverify = 0UL;
  int block_started = 0, block_ended = 0;
  double t0 = now();
  t_start = t0; t_ingest = t_bulk = t_sv_last = 0.0;
  for(;;) {
    int progress = 0;
    if( fec_i<fec_cnt && !bank_dead[ 1 ] ) {
      fd_sched_fec_t fec[ 1 ];
      memset( fec, 0, sizeof(fec) );
      fec->bank_idx          = 1UL;
      fec->parent_bank_idx   = 0UL;
      fec->slot              = 1UL;
      fec->parent_slot       = 0UL;
      fec->fec               = &fecs[ fec_i ];
      fec->shred_cnt         = 32U;
      fec->is_last_in_batch  = last_in_batch[ fec_i ] ? 1U : 0U;
      fec->is_last_in_block  = fec_i==fec_cnt-1UL ? 1U : 0U;
      fec->is_first_in_block = fec_i==0UL ? 1U : 0U;
      if( fd_sched_fec_can_ingest( sched, fec ) ) {
        double ti = now();
        FD_TEST( fd_sched_fec_ingest( sched, fec ) );
        t_ingest += now() - ti;
        fec_i++;
        progress = 1;
      }
    }
    if( mode!=MODE_EXEC ) { double tb = now(); progress |= bulk_sigverify( sched, bulk, mode, batch_min, batch_max ); t_bulk += now() - tb; }

    fd_sched_task_t task[ 1 ];
    if( fd_sched_task_next_ready( sched, task ) ) {
      progress = 1;
      switch( task->task_type ) {
        case FD_SCHED_TT_BLOCK_START:
          block_started = 1;
          fd_sched_task_done( sched, FD_SCHED_TT_BLOCK_START, ULONG_MAX, ULONG_MAX );
          break;
        case FD_SCHED_TT_BLOCK_END:
          block_ended = 1;
          fd_sched_task_done( sched, FD_SCHED_TT_BLOCK_END, ULONG_MAX, ULONG_MAX );
          break;
        case FD_SCHED_TT_TXN_EXEC:
          FD_TEST( pend[ task->txn_exec->exec_idx ].type==FD_SCHED_TT_NULL );
          pend[ task->txn_exec->exec_idx ].type    = FD_SCHED_TT_TXN_EXEC;
          pend[ task->txn_exec->exec_idx ].txn_idx = task->txn_exec->txn_idx;
          bank_refcnt[ task->txn_exec->bank_idx ]++;
          pend_cnt++; tasks_exec++;
          break;
        case FD_SCHED_TT_TXN_SIGVERIFY:
          FD_TEST( pend[ task->txn_sigverify->exec_idx ].type==FD_SCHED_TT_NULL );
          pend[ task->txn_sigverify->exec_idx ].type    = FD_SCHED_TT_TXN_SIGVERIFY;
          pend[ task->txn_sigverify->exec_idx ].txn_idx = task->txn_sigverify->txn_idx;
          bank_refcnt[ task->txn_sigverify->bank_idx ]++;
          pend_cnt++; tasks_sigverify++;
          break;
        default: FD_LOG_ERR(( "unexpected task type %lu", task->task_type ));
      }
    } else if( pend_cnt ) {
      /* an emulated exec tile finishes its task (process_exec_task_done) */
      for( ulong s=0UL; s<exec_cnt; s++ ) {
        ulong k = (rr+s)%exec_cnt;
        if( pend[ k ].type==FD_SCHED_TT_NULL ) continue;
        ulong type = pend[ k ].type, txn_idx = pend[ k ].txn_idx;
        pend[ k ].type = FD_SCHED_TT_NULL;
        pend_cnt--;
        rr = k+1UL;
        bank_refcnt[ 1 ]--;
        if( type==FD_SCHED_TT_TXN_SIGVERIFY ) {
          fd_txn_p_t * txn_p = fd_sched_get_txn( sched, txn_idx );
          int res = txn_verify_ref( txn_p );
          sigs_exec += TXN( txn_p )->signature_cnt;
          record( sched, txn_idx, res, 1 );
          sigverify_failed( sched, 1UL, res );
          t_sv_last = now() - t_start;
        }
        fd_sched_task_done( sched, type, txn_idx, k );
        break;
      }
      progress = 1;
    }
    if( block_ended ) break;
    if( bank_dead[ 1 ] && !pend_cnt && !bulk->cnt ) break;     /* abandoned and drained */
    if( !progress ) {
      if( ++idle>(1UL<<24) ) FD_LOG_ERR(( "stalled: fec %lu/%lu, pending %lu, bulk %lu", fec_i, fec_cnt, pend_cnt, bulk->cnt ));
    } else idle = 0UL;
  }
  double dt = now() - t0;
  if( !bank_dead[ 1 ] ) FD_TEST( !pend_cnt && !bulk->cnt && bank_refcnt[ 1 ]==0UL );

  FILE * o = fopen( argv[4], "wb" ); FD_TEST( o );
  FD_TEST( fwrite( "FDR1", 1, 4, o )==4 && fwrite( &rec_cnt, 8, 1, o )==1 &&
           fwrite( recs, sizeof(rec_t), rec_cnt, o )==rec_cnt );
  fclose( o );
  char svc_extra[ 160 ] = "";
#if FD_HAS_HIP_SVC
  if( mode==MODE_SVC ) {
    ulong threads, dev_fds; svc_client_census( &threads, &dev_fds );
    snprintf( svc_extra, sizeof(svc_extra), ", \"threads\": %lu, \"dev_fds\": %lu, \"svc_requests\": %lu, \"svc_sigs\": %lu",
              threads, dev_fds, bulk->svc->c->reqs_posted, bulk->svc->sigs );
  }
#endif
  printf( "{\"mode\": \"%s\", \"record\": %d, \"exec_cnt\": %lu, \"fec_cnt\": %lu, \"fec_ingested\": %lu, "
          "\"sigverified\": %lu, \"tasks_exec\": %lu, \"tasks_sigverify\": %lu, \"bulk_batches\": %lu, "
          "\"bulk_max\": %lu, \"sigs_exec\": %lu, \"sigs_bulk\": %lu, \"block_started\": %d, \"block_ended\": %d, "
          "\"dead\": %d, \"refcnt\": %lu, \"seconds\": %.6f, \"batch_max\": %lu, \"batch_min\": %lu, "
          "\"ingest_s\": %.6f, \"bulk_s\": %.6f, \"sigverify_done_s\": %.6f%s}\n",
          argv[1], record_mode, exec_cnt, fec_cnt, fec_i, rec_cnt, tasks_exec, tasks_sigverify, batches_bulk, bulk_max,
          sigs_exec, sigs_bulk, block_started, block_ended, bank_dead[ 1 ], bank_refcnt[ 1 ], dt, batch_max, batch_min,
          t_ingest, t_bulk, t_sv_last, svc_extra );
  fflush( stdout );
#if FD_HAS_HIP
  if( hip ) {
    fd_replay_hip_delete( bulk->replay ); fd_ed25519_hip_ctx_delete( hip );
    fd_ed25519_hip_host_free( bulk->pool ); fd_ed25519_hip_host_free( bulk->desc ); fd_ed25519_hip_host_free( bulk->result );
    bulk->result = NULL;
  }
#endif
  free( bulk->result ); free( bulk->txn_idx ); free( recs ); free( fecs ); free( last_in_batch );
  return 0;
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  if( argc!=2 && argc<6 ) {
    fprintf( stderr, "usage: %s fecs.bin exec|claim|skip|hip|svc exec_cnt record out.bin [batch_max] [batch_min]\n"
                     "       %s jobs.txt   (one job per line, same fields)\n", argv[0], argv[0] );
    return 2;
  }
  ulong fp = fd_sched_footprint( BANK_CNT );
  ulong const huge = 1UL<<21;
  void * mem = mmap( NULL, fp + huge, PROT_READ|PROT_WRITE, MAP_PRIVATE|MAP_ANONYMOUS|MAP_NORESERVE, -1, 0 );
  FD_TEST( mem!=MAP_FAILED );
  sched_mem = (void *)fd_ulong_align_up( (ulong)mem, huge );
  (void)madvise( sched_mem, fd_ulong_align_up( fp, huge ), MADV_HUGEPAGE );

  static uchar sha_mem[ FD_TXN_ACTUAL_SIG_MAX ][ sizeof(fd_sha512_t) ] __attribute__((aligned(FD_SHA512_ALIGN)));
  for( ulong k=0UL; k<FD_TXN_ACTUAL_SIG_MAX; k++ ) shas[ k ] = fd_sha512_join( fd_sha512_new( sha_mem[ k ] ) );

  if( argc>=6 ) {
    int rc = run_job( argv+1, argc-1 );
#if FD_HAS_HIP_SVC
    svc_client_done();
#endif
    return rc;
  }
  FILE * jf = fopen( argv[1], "r" ); FD_TEST( jf );
  char line[ 4096 ];
  while( fgets( line, sizeof(line), jf ) ) {
    char * tok[ 8 ]; int n = 0;
    for( char * t = strtok( line, " \t\n" ); t && n<8; t = strtok( NULL, " \t\n" ) ) tok[ n++ ] = t;
    if( !n ) continue;
    int rc = run_job( tok, n );
    if( rc ) return rc;
  }
  fclose( jf );
#if FD_HAS_HIP_SVC
  svc_client_done();
#endif
  return 0;
}
