/* fec_run.c -- the reference's FEC resolver (src/disco/shred/fd_fec_resolver.c)
   with integration/fd_fec_resolver_hip.patch, fed a shred stream made by the
   reference's own shredder (src/disco/shred/fd_shredder.c).

     fec_run <out.bin> [sets] [seed] [window]

   integration/Makefile builds it twice from the same sources:
     _build/fec_run_ref   the patch with FD_HAS_HIP off: the reference's add_shred
     _build/fec_run       FD_HAS_HIP: the engine attached (fd_fec_resolver_hip_attach),
                          every window of shreds handed to fd_fec_resolver_hip_preverify
                          before add_shred takes them one at a time
   Both write one record per shred -- add_shred's return value and, for a
   shred that completes a FEC set, the out shred's slot and fec_set_idx, the
   set's Merkle root and a hash of its data and parity shreds -- so their
   files compare byte for byte (tests/test_gpu_fec.py).

   Stream: `sets` FEC sets (default 2048) cut by the shredder from random
   entry batches, one slot per batch, chained Merkle roots on even slots,
   signed with the leader key of `seed`.  Faults: every 7th set is signed
   by another key (its root verify fails: every shred rejected), every 11th
   has a bit of its first data shred's payload flipped (that shred's root
   is not the set's: rejected, the next shred starts the set), every 13th
   has a corrupted signature on every shred; 1 in 5 parity shreds are
   dropped and the shreds are shuffled within windows of `window` (default
   512).

   The FD_HAS_HIP build also checks every root the GPU verified against the
   reference's own fd_ed25519_verify on the same three inputs (codes must be
   equal), and reports the resolver's table hits (add_shred took the GPU's
   code) and core verifies.

     _build/fec_run_svc   FD_HAS_HIP_SVC: no HIP in the process; the resolver
                          is a client of the GPU tile's service
                          (fd_fec_resolver_hip_attach_svc, integration/svc_client.h:
                          SVC_CLIENT_SHM names the run, svc_tile_run host or
                          produce with SVC_RUN_CLIENTS); the same checks, the
                          codes compared by verdict (the service's contexts
                          give the AVX-512 build's error codes, this
                          process's reference verify the portable build's),
                          and the process's threads and device fds. */

#include "../../util/fd_util.h"
#include "../../ballet/shred/fd_shred.h"
#include "../../ballet/ed25519/fd_ed25519.h"
#include "fd_shredder.h"
#include "../metrics/fd_metrics.h"
#include FEC_SRC
#include <stdio.h>
#include <stdlib.h>
#if FD_HAS_HIP_SVC
#include "svc_client.h"
#endif

#if defined(fd_boot)
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

#define SHRED_VER ((ushort)6051)
#define MAX_IDX   (32768UL)
#define DEPTH     (64UL)
#define PARTIAL   (4UL)
#define COMPLETE  (4UL)
#define DONE      (4096UL)
#define SETS_MEM  (DEPTH+PARTIAL+COMPLETE)

typedef struct { fd_sha512_t sha[1]; uchar const * prv; uchar const * pub; } signer_t;

static void
sign_root( void * _s, uchar * sig, uchar const * root ) {
  signer_t * s = (signer_t *)_s;
  fd_ed25519_sign( sig, root, 32UL, s->pub, s->prv, s->sha );
}

static uchar *
set_mem( fd_fec_set_t * set, uchar * p ) {
  for( ulong j=0UL; j<FD_REEDSOL_DATA_SHREDS_MAX;   j++ ) { set->data_shreds  [ j ] = p; p += 2048UL; }
  for( ulong j=0UL; j<FD_REEDSOL_PARITY_SHREDS_MAX; j++ ) { set->parity_shreds[ j ] = p; p += 2048UL; }
  return p;
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  static uchar metrics[ FD_METRICS_FOOTPRINT( 0, 0 ) ] __attribute__((aligned(FD_METRICS_ALIGN)));
  fd_metrics_register( fd_metrics_new( metrics, 0UL, 0UL ) );    /* add_shred counts into the tile's metrics */
  if( argc<2 ) { fprintf( stderr, "usage: %s <out.bin> [sets] [seed] [window]\n", argv[0] ); return 2; }
  ulong sets_want = argc>2 ? strtoul( argv[2], NULL, 0 ) : 2048UL;
  ulong seed      = argc>3 ? strtoul( argv[3], NULL, 0 ) : 0x5eedfecUL;
  ulong window    = argc>4 ? strtoul( argv[4], NULL, 0 ) : 512UL;
  FD_TEST( sets_want>=1UL && window>=1UL );

  fd_rng_t _rng[1]; fd_rng_t * rng = fd_rng_join( fd_rng_new( _rng, (uint)seed, seed>>32 ) );
  uchar prv[ 2 ][ 32 ], pub[ 2 ][ 32 ];
  fd_sha512_t sha[1]; FD_TEST( fd_sha512_join( fd_sha512_new( sha ) ) );
  for( ulong k=0UL; k<2UL; k++ ) {
    for( ulong b=0UL; b<32UL; b++ ) prv[ k ][ b ] = fd_rng_uchar( rng );
    FD_TEST( fd_ed25519_public_from_private( pub[ k ], prv[ k ], sha ) );
  }
  signer_t sg[ 2 ];
  fd_shredder_t * shredder[ 2 ];
  static fd_shredder_t shredder_mem[ 2 ];
  for( ulong k=0UL; k<2UL; k++ ) {
    FD_TEST( fd_sha512_join( fd_sha512_new( sg[ k ].sha ) ) );
    sg[ k ].prv = prv[ k ]; sg[ k ].pub = pub[ k ];
    shredder[ k ] = fd_shredder_join( fd_shredder_new( &shredder_mem[ k ], sign_root, &sg[ k ] ) );
    FD_TEST( shredder[ k ] );
    fd_shredder_set_shred_version( shredder[ k ], SHRED_VER );
  }

  /* the stream: every shred of every set (1 in 5 parity shreds dropped), the faults, then the shuffle */
  ulong   cap    = sets_want*(FD_REEDSOL_DATA_SHREDS_MAX+FD_REEDSOL_PARITY_SHREDS_MAX);
  uchar * pool   = malloc( cap*FD_SHRED_MAX_SZ );
  ulong * sz     = malloc( cap*sizeof(ulong) );
  uchar * tmp    = malloc( 2048UL*(FD_REEDSOL_DATA_SHREDS_MAX+FD_REEDSOL_PARITY_SHREDS_MAX) );
  uchar * batch  = malloc( 1UL<<17 );
  FD_TEST( pool && sz && tmp && batch );
  fd_fec_set_t tmp_set[1]; set_mem( tmp_set, tmp );
  ulong cnt = 0UL, set_no = 0UL;
  uchar chained[ 32 ] = { 0 };
#define PUT_SHRED( p, psz ) do {                                                    \
    ulong _sz = (psz);                                                              \
    FD_TEST( cnt<cap && _sz<=FD_SHRED_MAX_SZ );                                     \
    memcpy( pool + cnt*FD_SHRED_MAX_SZ, (p), _sz ); sz[ cnt++ ] = _sz; } while(0)
  for( ulong slot=1UL; set_no<sets_want; slot++ ) {
    fd_shredder_t * sh  = shredder[ (slot%7UL)==6UL ];            /* the whole slot signed by the other key */
    ulong           bsz = 1000UL + fd_rng_ulong_roll( rng, 90000UL );
    for( ulong b=0UL; b<bsz; b++ ) batch[ b ] = fd_rng_uchar( rng );
    fd_entry_batch_meta_t meta[1]; memset( meta, 0, sizeof(meta) ); meta->block_complete = 1; meta->parent_offset = 1UL;
    FD_TEST( fd_shredder_init_batch( sh, batch, bsz, slot, meta ) );
    fd_fec_set_t * set;
    while( set_no<sets_want && ( set = fd_shredder_next_fec_set( sh, tmp_set, (slot&1UL) ? NULL : chained, NULL ) ) ) {
      ulong first = cnt;
      for( ulong j=0UL; j<set->data_shred_cnt;   j++ ) PUT_SHRED( set->data_shreds[ j ], FD_SHRED_MIN_SZ );
      for( ulong j=0UL; j<set->parity_shred_cnt; j++ ) if( fd_rng_uint_roll( rng, 5U ) ) PUT_SHRED( set->parity_shreds[ j ], FD_SHRED_MAX_SZ );
      if( ( set_no%11UL )==10UL ) pool[ first*FD_SHRED_MAX_SZ + FD_SHRED_DATA_HEADER_SZ + 17UL ] ^= (uchar)0x10;
      if( ( set_no%13UL )==12UL ) for( ulong j=first; j<cnt; j++ ) pool[ j*FD_SHRED_MAX_SZ + 5UL ] ^= (uchar)0x01;
      set_no++;
    }
    FD_TEST( fd_shredder_fini_batch( sh ) );
  }
#undef PUT_SHRED
  ulong * order = malloc( cnt*sizeof(ulong) );
  FD_TEST( order );
  for( ulong i=0UL; i<cnt; i++ ) order[ i ] = i;
  for( ulong w0=0UL; w0<cnt; w0+=window ) {                        /* shuffle within each window */
    ulong n = fd_ulong_min( window, cnt-w0 );
    for( ulong i=n-1UL; i>0UL; i-- ) { ulong j = fd_rng_ulong_roll( rng, i+1UL ); ulong t = order[ w0+i ]; order[ w0+i ] = order[ w0+j ]; order[ w0+j ] = t; }
  }

  /* the resolver (test_fec_resolver.c's setup, larger) */
  uchar * smem = malloc( SETS_MEM*2048UL*(FD_REEDSOL_DATA_SHREDS_MAX+FD_REEDSOL_PARITY_SHREDS_MAX) );
  static fd_fec_set_t out_sets[ SETS_MEM ];
  FD_TEST( smem );
  for( ulong i=0UL; i<SETS_MEM; i++ ) set_mem( out_sets+i, smem + i*2048UL*(FD_REEDSOL_DATA_SHREDS_MAX+FD_REEDSOL_PARITY_SHREDS_MAX) );
  ulong foot = fd_fec_resolver_footprint( DEPTH, PARTIAL, COMPLETE, DONE );
  void * rmem = aligned_alloc( FD_FEC_RESOLVER_ALIGN, fd_ulong_align_up( foot, FD_FEC_RESOLVER_ALIGN ) );
  FD_TEST( foot && rmem );
  fd_fec_resolver_t * r = fd_fec_resolver_join( fd_fec_resolver_new( rmem, NULL, NULL, DEPTH, PARTIAL, COMPLETE, DONE, out_sets, MAX_IDX ) );
  FD_TEST( r );
  fd_fec_resolver_set_shred_version( r, SHRED_VER );
#if FD_HAS_HIP
  fd_ed25519_hip_ctx_t * hip = fd_ed25519_hip_ctx_new( 0, FD_FEC_RESOLVER_HIP_BATCH_MAX );
  FD_TEST( hip );
  fd_ed25519_hip_set_errmode( hip, FD_ED25519_HIP_ERRMODE_REF );   /* codes of the reference's portable build, linked here */
  FD_TEST( !fd_fec_resolver_hip_attach( r, hip ) );
  FD_TEST( window<=FD_FEC_RESOLVER_HIP_BATCH_MAX );               /* one launch per window: its roots are checked below */
  ulong checked = 0UL, code_bad = 0UL;
#elif FD_HAS_HIP_SVC
  ulong svc_t;
  fd_verify_svc_seg_t * svc_seg = svc_client_attach( &svc_t );
  void * svc_mem = aligned_alloc( 128UL, fd_ulong_align_up( fd_fec_resolver_hip_svc_footprint(), 128UL ) );
  FD_TEST( svc_mem && !fd_fec_resolver_hip_attach_svc( r, svc_seg, svc_t, svc_mem ) );
  FD_TEST( window<=FD_FEC_RESOLVER_HIP_BATCH_MAX );
  ulong checked = 0UL, code_bad = 0UL, code_diff = 0UL;
#endif

  FILE * out = fopen( argv[1], "wb" );
  FD_TEST( out );
  fd_shred_t const * parsed[ 4096 ];
  ulong              psz   [ 4096 ];
  uchar const *      ppub  [ 4096 ];
  FD_TEST( window<=4096UL );
  ulong rv_cnt[ 4 ] = { 0UL };
  long  t_add = 0L;
  for( ulong w0=0UL; w0<cnt; w0+=window ) {
    ulong n = fd_ulong_min( window, cnt-w0 );
    for( ulong j=0UL; j<n; j++ ) {
      ulong i = order[ w0+j ];
      parsed[ j ] = fd_shred_parse( pool + i*FD_SHRED_MAX_SZ, sz[ i ] );
      if( FD_UNLIKELY( !parsed[ j ] ) ) FD_LOG_ERR(( "shred %lu (stream %lu) sz %lu variant %02x data.size %u does not parse", w0+j, i, sz[ i ], (uint)pool[ i*FD_SHRED_MAX_SZ+64 ], (uint)*(ushort *)( pool + i*FD_SHRED_MAX_SZ + 86 ) ));
      psz[ j ] = sz[ i ]; ppub[ j ] = pub[ 0 ];
    }
    long t0 = fd_log_wallclock();
#if FD_HAS_HIP
    ulong m = fd_fec_resolver_hip_preverify( r, parsed, psz, ppub, n );
    t_add += fd_log_wallclock() - t0;
    for( ulong j=0UL; j<m; j++ ) {                                 /* the GPU's codes against the reference's verify */
      int ref = fd_ed25519_verify( r->hip_roots + 32UL*j, 32UL, r->hip_sigs + 64UL*j, r->hip_pubs + 32UL*j, sha );
      code_bad += ref!=(int)r->hip_codes[ j ];
    }
    checked += m;
    t0 = fd_log_wallclock();
#elif FD_HAS_HIP_SVC
    ulong m = fd_fec_resolver_hip_preverify( r, parsed, psz, ppub, n );
    t_add += fd_log_wallclock() - t0;
    for( ulong j=0UL; j<m; j++ ) {                                 /* the service's verdicts against the reference's verify */
      int ref = fd_ed25519_verify( r->hip_roots + 32UL*j, 32UL, r->hip_sigs + 64UL*j, r->hip_pubs + 32UL*j, sha );
      code_bad  += ( ref==FD_ED25519_SUCCESS )!=( (int)r->hip_codes[ j ]==FD_ED25519_SUCCESS );
      code_diff += ref!=(int)r->hip_codes[ j ];
    }
    checked += m;
    t0 = fd_log_wallclock();
#endif
    for( ulong j=0UL; j<n; j++ ) {
      fd_fec_set_t const * out_fec = NULL; fd_shred_t const * out_shred = NULL;
      fd_bmtree_node_t out_root[1]; fd_fec_resolver_spilled_t spilled; memset( &spilled, 0, sizeof(spilled) );
      int rv = fd_fec_resolver_add_shred( r, parsed[ j ], psz[ j ], ppub[ j ], &out_fec, &out_shred, out_root, &spilled );
      rv_cnt[ rv + FD_FEC_RESOLVER_ADD_SHRED_RETVAL_OFF ]++;
      schar c = (schar)rv;
      FD_TEST( fwrite( &c, 1UL, 1UL, out )==1UL );
      if( rv==FD_FEC_RESOLVER_SHRED_COMPLETES ) {
        ulong h = 0x5eedfecUL;
        for( ulong d=0UL; d<out_fec->data_shred_cnt;   d++ ) h = fd_hash( h, out_fec->data_shreds  [ d ], FD_SHRED_MIN_SZ );
        for( ulong d=0UL; d<out_fec->parity_shred_cnt; d++ ) h = fd_hash( h, out_fec->parity_shreds[ d ], FD_SHRED_MAX_SZ );
        ulong rec[ 3 ] = { out_shred->slot, (ulong)out_shred->fec_set_idx, h };
        FD_TEST( fwrite( rec, sizeof(rec), 1UL, out )==1UL );
        FD_TEST( fwrite( out_root->hash, 32UL, 1UL, out )==1UL );
      }
    }
    t_add += fd_log_wallclock() - t0;
  }
  FD_TEST( !fclose( out ) );
  printf( "{\"shreds\": %lu, \"sets\": %lu, \"rejected\": %lu, \"ignored\": %lu, \"okay\": %lu, \"completes\": %lu, "
          "\"resolver_s\": %.6f", cnt, set_no, rv_cnt[ 0 ], rv_cnt[ 1 ], rv_cnt[ 2 ], rv_cnt[ 3 ], (double)t_add*1e-9 );
#if FD_HAS_HIP
  ulong st[ 4 ]; fd_fec_resolver_hip_stats( r, st );
  printf( ", \"hip\": 1, \"roots_verified\": %lu, \"launches\": %lu, \"table_hits\": %lu, \"core_verifies\": %lu, "
          "\"roots_checked\": %lu, \"code_mismatch\": %lu", st[ 0 ], st[ 1 ], st[ 2 ], st[ 3 ], checked, code_bad );
#elif FD_HAS_HIP_SVC
  ulong st[ 4 ]; fd_fec_resolver_hip_stats( r, st );
  ulong threads, dev_fds; svc_client_census( &threads, &dev_fds );
  printf( ", \"hip\": 2, \"roots_verified\": %lu, \"launches\": %lu, \"table_hits\": %lu, \"core_verifies\": %lu, "
          "\"roots_checked\": %lu, \"code_mismatch\": %lu, \"code_diff\": %lu, \"threads\": %lu, \"dev_fds\": %lu, "
          "\"svc_requests\": %lu", st[ 0 ], st[ 1 ], st[ 2 ], st[ 3 ], checked, code_bad, code_diff, threads, dev_fds,
          r->hip_svc->reqs_posted );
  svc_client_done();
#else
  printf( ", \"hip\": 0" );
#endif
  printf( "}\n" );
  return 0;
}
