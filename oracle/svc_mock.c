/* svc_mock.c -- TEST INFRASTRUCTURE ONLY (repo-owned).

   A CPU stand-in for the GPU tile of the service-mode verify stage
   (integration/svc_run.c): it answers the verify tiles' requests through
   the same segment (include/fd_verify_svc.h) with the reference's own code
   -- before_frag's share, during_frag's checks and copy (or a gossip vote's
   conversion), fd_txn_parse, fd_hash of sig0, and the portable backend's
   fd_ed25519_verify_batch_single_msg (src/ballet/ed25519/fd_ed25519_user.c,
   compiled from the reference by oracle/Makefile) -- and writes flushed
   frags into the tiles' out dcaches.  It lets the CPU suite exercise the
   tile side of the protocol (credits, flush order, publish order, metrics,
   the overrun checks) without a GPU; the product's GPU tile is
   firedancer_amd/csrc/fd_verify_svc.hip, which never uses this file.

     svc_mock <shm> <gpu (ignored)>       (same command line as svc_run)

   SVC_MOCK_INGEST=us: answer in two steps as the GPU tile does -- copy a
   posted request's frags (the link's bytes) into staging and mark it
   INGESTED, then, at least `us` microseconds later, parse and verify from
   staging only and mark it RESULTS (the tile returns the link's credits in
   between); default: both at once, straight to RESULTS.

   Client tiles (the segment's tiles after the run's tile_cnt verify tiles,
   integration/svc_client.h) post FD_VERIFY_SVC_REQ_SIGS records: each is
   answered with the reference's fd_ed25519_verify. */

#include "../../tango/mcache/fd_mcache.h"
#include "../../tango/dcache/fd_dcache.h"
#include "../../ballet/txn/fd_txn.h"
#include "../../ballet/ed25519/fd_ed25519.h"
#include "../fd_txn_m.h"
#include "../quic/fd_tpu.h"
#include "../../flamenco/gossip/fd_gossip_types.h"
#include "fd_verify_svc.h"
#include "../integration/svc_run.h"
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#if defined(fd_boot)
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

#define STAGE_SZ (2176UL)

static uchar * stage;                          /* tile x slot x slot_cap staging frags */
static fd_sha512_t * shas[ 16 ];
typedef struct { uchar flags; uchar kind; ushort sz; uint tsorig; } meta_t;
static meta_t * meta;                          /* per staging frag: what the ingest saw */

static uchar *
stage_of( fd_verify_svc_seg_t * s, ulong t, ulong slot, ulong j ) {
  return stage + ( ( t*s->req_depth + slot )*s->slot_cap + j )*STAGE_SZ;
}

/* the ingest: before_frag's share, during_frag's checks and copy (or a
   gossip vote's conversion) into staging; nothing after this reads the link */
static void
ingest( svc_run_hdr_t * hdr, uchar * base, fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  fd_verify_svc_req_t * q = fd_verify_svc_req( s, t, slot );
  for( ulong j=0UL; j<q->n; j++ ) {
    meta_t * m = &meta[ ( t*s->req_depth + slot )*s->slot_cap + j ];
    uchar * dst = stage_of( s, t, slot, j );
    ulong sz = 0UL, kind = 0UL;                                  /* FD_VERIFY_HIP_IN_QUIC */
    int   ok = 1;
    uchar const * src = NULL;
    m->flags = 0; m->tsorig = 0U; m->sz = 0;
    if( q->kind==FD_VERIFY_SVC_REQ_SIGS ) {                     /* a client's signature record, as it stands */
      sz = fd_verify_svc_frag_sz( s, t, slot )[ j ];
      m->kind = 0xff;
      if( sz<FD_VERIFY_SVC_SIG_HDR_SZ || sz>FD_VERIFY_SVC_FRAG_STRIDE ) { m->flags = FD_VERIFY_SVC_RES_BAD; continue; }
      memcpy( dst, fd_verify_svc_frag( s, t, slot ) + j*FD_VERIFY_SVC_FRAG_STRIDE, sz );
      m->sz = (ushort)sz;
      continue;
    }
    if( q->kind==FD_VERIFY_SVC_REQ_RANGE ) {
      ulong first = fd_verify_svc_range_first( q->seq0, q->rr_cnt, q->rr_idx ), seq = first + j*q->rr_cnt;
      fd_frag_meta_t const * mc   = fd_mcache_join( base + hdr->mcache_off[ q->link ] );
      ulong                  dpth = fd_mcache_depth( mc );
      fd_frag_meta_t const * line = mc + fd_mcache_line_idx( seq, dpth );
      uchar const *          dc   = fd_dcache_join( base + hdr->dcache_off[ q->link ] );
      ulong chunk = line->chunk; sz = line->sz; m->tsorig = line->tsorig;
      ok  = line->seq==seq && chunk>=fd_dcache_compact_chunk0( base, dc ) &&
            chunk<=fd_dcache_compact_wmark( base, dc, FD_TPU_REASM_MTU ) && sz<=FD_TPU_RAW_MTU;
      src = (uchar const *)fd_chunk_to_laddr_const( base, chunk );
    } else {
      src  = fd_verify_svc_frag( s, t, slot ) + j*FD_VERIFY_SVC_FRAG_STRIDE;
      sz   = fd_verify_svc_frag_sz( s, t, slot )[ j ];
      kind = fd_verify_svc_frag_kind( s, t, slot )[ j ];
      ok   = sz<=( kind==2UL ? 2048UL : FD_TPU_RAW_MTU );
    }
    m->kind = (uchar)kind;
    if( !ok ) { m->flags = FD_VERIFY_SVC_RES_BAD; continue; }
    fd_txn_m_t * txnm = (fd_txn_m_t *)dst;
    if( kind==2UL ) {                                            /* during_frag's vote conversion, fd_verify_tile.c:86-97 */
      fd_gossip_update_message_t const * msg = (fd_gossip_update_message_t const *)src;
      memset( dst, 0, sizeof(fd_txn_m_t) );
      if( msg->vote.txn_sz>FD_TPU_MTU ) { m->flags = FD_VERIFY_SVC_RES_BAD; continue; }
      txnm->payload_sz = (ushort)msg->vote.txn_sz; txnm->block_engine.bundle_id = 0UL;
      txnm->source_ipv4 = msg->vote.socket.addr; txnm->source_tpu = FD_TXN_M_TPU_SOURCE_GOSSIP;
      memcpy( fd_txn_m_payload( txnm ), msg->vote.txn, msg->vote.txn_sz );
    } else {
      memset( dst, 0, STAGE_SZ );
      memcpy( dst, src, sz );
      if( txnm->payload_sz>FD_TPU_MTU ) { m->flags = FD_VERIFY_SVC_RES_BAD; continue; }
      if( sz<sizeof(fd_txn_m_t) + txnm->payload_sz ) m->flags = FD_VERIFY_SVC_RES_HOST;
    }
  }
}

/* the verify, from staging: fd_txn_parse, the sig0 tag, the reference's
   fd_ed25519_verify_batch_single_msg */
static void
answer( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  fd_verify_svc_req_t * q   = fd_verify_svc_req( s, t, slot );
  fd_verify_svc_res_t * res = fd_verify_svc_res( s, t, slot );
  for( ulong j=0UL; j<q->n; j++ ) {
    meta_t const * m = &meta[ ( t*s->req_depth + slot )*s->slot_cap + j ];
    fd_verify_svc_res_t r; memset( &r, 0, sizeof(r) );
    r.flags = m->flags; r.tsorig = m->tsorig;
    if( q->kind==FD_VERIFY_SVC_REQ_SIGS ) {                     /* fd_ed25519_verify of the record (the reference's) */
      if( m->flags & FD_VERIFY_SVC_RES_BAD ) { r.code = (schar)FD_ED25519_ERR_SIG; res[ j ] = r; continue; }
      uchar const * rec = stage_of( s, t, slot, j );
      ulong msz = (ulong)m->sz - FD_VERIFY_SVC_SIG_HDR_SZ;
      r.code = (schar)fd_ed25519_verify( rec + FD_VERIFY_SVC_SIG_HDR_SZ, msz, rec, rec + 64UL, shas[ 0 ] );
      r.sig_cnt = 1; r.payload_sz = (ushort)msz;
      res[ j ] = r;
      continue;
    }
    if( m->flags & FD_VERIFY_SVC_RES_BAD ) { res[ j ] = r; continue; }
    fd_txn_m_t * txnm = (fd_txn_m_t *)stage_of( s, t, slot, j );
    fd_txn_t * txnt = fd_txn_m_txn_t( txnm );
    txnm->txn_t_sz = (ushort)fd_txn_parse( fd_txn_m_payload( txnm ), txnm->payload_sz, txnt, NULL );
    r.txn_t_sz = txnm->txn_t_sz; r.payload_sz = txnm->payload_sz; r.bundle_id = txnm->block_engine.bundle_id;
    if( r.txn_t_sz ) {
      uchar const * pay = fd_txn_m_payload( txnm );
      r.tag     = fd_hash( q->seed, pay + txnt->signature_off, 64UL );
      r.sig_cnt = txnt->signature_cnt;
      r.code    = (schar)fd_ed25519_verify_batch_single_msg( pay + txnt->message_off, (ulong)txnm->payload_sz - txnt->message_off,
                                                              pay + txnt->signature_off, pay + txnt->acct_addr_off, shas,
                                                              txnt->signature_cnt );
    }
    res[ j ] = r;
  }
  q->batch_frags = q->n;
  fd_verify_svc_st( &q->state, FD_VERIFY_SVC_RESULTS );
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  if( argc<3 ) { fprintf( stderr, "usage: %s <shm> <gpu>\n", argv[0] ); return 2; }
  int fd = open( argv[1], O_RDWR );
  if( fd<0 ) FD_LOG_ERR(( "open(%s) failed", argv[1] ));
  svc_run_hdr_t h;
  if( pread( fd, &h, sizeof(h), 0 )!=(long)sizeof(h) || h.magic!=SVC_RUN_MAGIC ) FD_LOG_ERR(( "not a svc_run segment" ));
  uchar * base = mmap( NULL, h.map_sz, PROT_READ|PROT_WRITE, MAP_SHARED, fd, 0 );
  FD_TEST( base!=MAP_FAILED );
  close( fd );
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;
  fd_verify_svc_seg_t * s = fd_verify_svc_join( base + hdr->svc_off );
  FD_TEST( s );
  stage = malloc( s->tile_cnt*s->req_depth*s->slot_cap*STAGE_SZ );
  meta  = malloc( s->tile_cnt*s->req_depth*s->slot_cap*sizeof(meta_t) );
  FD_TEST( stage && meta );
  char const * ing_env = getenv( "SVC_MOCK_INGEST" );
  long const   ing_ns  = ing_env ? 1000L*strtol( ing_env, NULL, 0 ) : -1L;   /* -1: straight to RESULTS */
  ulong vtake[ FD_VERIFY_SVC_TILE_MAX ] = { 0UL };                  /* requests verified (ingest mode) */
  long  ing_at[ FD_VERIFY_SVC_TILE_MAX ][ 256 ];                    /* when each slot was ingested */
  for( ulong k=0UL; k<16UL; k++ ) shas[ k ] = fd_sha512_join( fd_sha512_new( aligned_alloc( FD_SHA512_ALIGN, FD_SHA512_FOOTPRINT ) ) );
  ulong take[ FD_VERIFY_SVC_TILE_MAX ] = { 0UL }, ftake[ FD_VERIFY_SVC_TILE_MAX ] = { 0UL };
  ulong st[ 8 ] = { 0UL };
  fd_verify_svc_st( &s->svc_state, FD_VERIFY_SVC_SVC_RUNNING );
  hdr->svc_ready = 1UL;
  while( !hdr->shutdown ) {
    int did = 0;
    for( ulong t=0UL; t<s->tile_cnt; t++ ) {
      for( ;; ) {
        ulong slot = take[ t ] & ( s->req_depth-1UL );
        fd_verify_svc_req_t * q = fd_verify_svc_req( s, t, slot );
        if( fd_verify_svc_ld( &q->state )!=FD_VERIFY_SVC_POSTED ) break;
        if( q->id+s->req_depth==take[ t ] ) break;               /* the slot's previous request, not yet verified */
        FD_TEST( q->id==take[ t ] );
        FD_TEST( ( t>=hdr->tile_cnt )==( q->kind==FD_VERIFY_SVC_REQ_SIGS ) );   /* clients post signature records only */
        ingest( hdr, base, s, t, slot );
        if( ing_ns<0L ) { answer( s, t, slot ); vtake[ t ]++; }
        else { fd_verify_svc_st( &q->state, FD_VERIFY_SVC_INGESTED ); ing_at[ t ][ slot ] = fd_log_wallclock(); }
        st[ 0 ]++; st[ 1 ] += q->n; st[ 2 ]++;
        take[ t ]++; did = 1;
      }
      while( vtake[ t ]<take[ t ] ) {                            /* ingest mode: verify after the delay, in order */
        ulong slot = vtake[ t ] & ( s->req_depth-1UL );
        if( fd_log_wallclock()-ing_at[ t ][ slot ]<ing_ns ) break;
        answer( s, t, slot );
        vtake[ t ]++; did = 1;
      }
      fd_verify_svc_tile_t * b = fd_verify_svc_tile( s, t );
      ulong post = fd_verify_svc_ld( &b->flush_post );
      if( t>=hdr->tile_cnt ) { FD_TEST( !post ); continue; }     /* a client: no out dcache, no flush */
      uchar * odc = fd_dcache_join( base + hdr->out_dcache_off[ t ] );
      ulong   osz = fd_dcache_data_sz( odc );
      while( ftake[ t ]<post ) {
        fd_verify_svc_flush_t const * f = &b->flush[ ftake[ t ] & ( FD_VERIFY_SVC_FLUSH_DEPTH-1UL ) ];
        fd_verify_svc_out_t const * out = fd_verify_svc_out( s, t, f->slot );
        for( ulong e=f->lo; e<f->hi; e++ ) {
          if( out[ e ].flags & FD_VERIFY_SVC_OUT_HOSTWRITTEN ) continue;
          uchar * d = (uchar *)fd_chunk_to_laddr( base, out[ e ].chunk );
          FD_TEST( d>=odc && d+out[ e ].sz<=odc+osz );
          memcpy( d, stage_of( s, t, f->slot, out[ e ].idx ), out[ e ].sz );
          st[ 5 ] += out[ e ].sz;
        }
        st[ 3 ]++; st[ 4 ] += f->hi - f->lo;
        ftake[ t ]++; did = 1;
        fd_verify_svc_st( &b->flush_done, ftake[ t ] );
      }
    }
    if( !did ) FD_SPIN_PAUSE();
  }
  for( ulong k=0UL; k<8UL; k++ ) hdr->svc_stats[ k ] = st[ k ];   /* no host-time stats */
  FD_COMPILER_MFENCE();
  hdr->svc_done = 1UL;
  return 0;
}
