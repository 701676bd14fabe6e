/* firedancer_amd/csrc/fd_ed25519_multi.cpp
 *
 * Multi-device engine (include/fd_ed25519_amd.h, fd_ed25519_amd_multi_*;
 * SURVEY.md s8 e).  Signatures are independent, so a batch is split into
 * contiguous shards, one per engine, each engine bound to one device and
 * driven by its own persistent host thread.  Nothing crosses between
 * devices: every shard's inputs go host -> its GPU, its verdicts GPU ->
 * host.  This is the engine-level form of the reference's horizontal
 * scaling, N verify tiles each with its own input link
 * (src/app/frank/fd_frank_init:67-80, src/app/fdctl/config/default.toml:
 * 79-81).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fd_ed25519_amd.h"
#include "../../include/fd_txn_amd.h"
#include "fd_ed25519_engine.h"

struct fd_ed25519_amd_multi {
  ulong                             ndev;
  std::vector<fd_ed25519_amd_t *>   eng;
  std::vector<std::thread>          th;
  std::mutex                        mu;
  std::condition_variable           cv_go, cv_done;
  ulong                             gen = 0, pending = 0;
  bool                              quit = false;
  std::function<int( ulong )>       job;
  std::vector<int>                  rc;
};

extern "C" void
fd_ed25519_amd_shard_range( ulong n, ulong ndev, ulong r, ulong * lo, ulong * hi ) {
  /* n*r/ndev without overflow for any n < 2^64 / 2^8 (ndev <= 256) */
  *lo = (ulong)(((unsigned __int128)n * r) / ndev);
  *hi = (ulong)(((unsigned __int128)n * (r + 1UL)) / ndev);
}

/* Engine r's thread: bound to its device's NUMA node (CPUs and memory,
   fd_numa.cpp), it creates the engine there (so the pinned staging it
   fills is node-local), then serves batches. */
static void
worker( fd_ed25519_amd_multi_t * m, ulong r, int device, ulong batch_max, ulong blob_max ) {
  (void)fd_amd_numa_bind_thread( device );
  fd_ed25519_amd_t * e = fd_ed25519_amd_new( device, batch_max, blob_max );
  {
    std::lock_guard<std::mutex> lk( m->mu );
    m->eng[r] = e;
    if( !--m->pending ) m->cv_done.notify_all();
  }
  ulong seen = 0;
  for( ;; ) {
    std::function<int( ulong )> job;
    {
      std::unique_lock<std::mutex> lk( m->mu );
      m->cv_go.wait( lk, [&]{ return m->quit || m->gen != seen; } );
      if( m->quit ) return;
      seen = m->gen;
      job = m->job;
    }
    int rc = job( r );
    {
      std::lock_guard<std::mutex> lk( m->mu );
      m->rc[r] = rc;
      if( !--m->pending ) m->cv_done.notify_all();
    }
  }
}

/* Run job(r) on every engine's thread; the first nonzero return code. */
static int
run_all( fd_ed25519_amd_multi_t * m, std::function<int( ulong )> job ) {
  {
    std::lock_guard<std::mutex> lk( m->mu );
    m->job = std::move( job );
    m->pending = m->ndev;
    m->gen++;
  }
  m->cv_go.notify_all();
  std::unique_lock<std::mutex> lk( m->mu );
  m->cv_done.wait( lk, [&]{ return !m->pending; } );
  for( ulong r=0; r<m->ndev; r++ ) if( m->rc[r] ) return m->rc[r];
  return FD_ED25519_AMD_OK;
}

extern "C" void
fd_ed25519_amd_multi_delete( fd_ed25519_amd_multi_t * m ) {
  if( !m ) return;
  {
    std::lock_guard<std::mutex> lk( m->mu );
    m->quit = true;
  }
  m->cv_go.notify_all();
  for( auto & t : m->th ) if( t.joinable() ) t.join();
  for( auto * e : m->eng ) if( e ) fd_ed25519_amd_delete( e );
  delete m;
}

extern "C" fd_ed25519_amd_multi_t *
fd_ed25519_amd_multi_new( int const * devices, ulong ndev, ulong batch_max, ulong blob_max ) {
  if( !devices || !ndev || ndev > 256UL ) return NULL;
  fd_ed25519_amd_multi_t * m = new fd_ed25519_amd_multi_t();
  m->ndev = ndev;
  m->rc.assign( ndev, 0 );
  m->eng.assign( ndev, NULL );
  m->pending = ndev;
  for( ulong r=0; r<ndev; r++ ) m->th.emplace_back( worker, m, r, devices[r], batch_max, blob_max );
  {
    std::unique_lock<std::mutex> lk( m->mu );
    m->cv_done.wait( lk, [&]{ return !m->pending; } );
  }
  for( ulong r=0; r<ndev; r++ ) if( !m->eng[r] ) { fd_ed25519_amd_multi_delete( m ); return NULL; }
  return m;
}

extern "C" ulong
fd_ed25519_amd_multi_ndev( fd_ed25519_amd_multi_t const * m ) {
  return m ? m->ndev : 0UL;
}

extern "C" int
fd_ed25519_amd_multi_verify_soa( fd_ed25519_amd_multi_t * m, ulong n, uchar const * pub, uchar const * sig,
                                 uint const * msg_off, uint const * msg_sz, uchar const * blob, ulong blob_sz,
                                 schar * err ) {
  if( !m || (n && (!pub || !sig || !msg_off || !msg_sz || !err)) ) return FD_ED25519_AMD_ERR_INVAL;
  /* validated once for the whole batch, so either every shard runs or none */
  ulong cap = m->eng[0]->blob_cap;
  for( ulong i=0; i<n; i++ )
    if( msg_sz[i] && ((ulong)msg_off[i] + msg_sz[i] > blob_sz || !blob || msg_sz[i] > cap) ) return FD_ED25519_AMD_ERR_INVAL;
  if( !n ) return FD_ED25519_AMD_OK;
  return run_all( m, [&]( ulong r ) -> int {
    ulong lo, hi;
    fd_ed25519_amd_shard_range( n, m->ndev, r, &lo, &hi );
    if( lo == hi ) return FD_ED25519_AMD_OK;
    return fd_ed25519_amd_verify_soa( m->eng[r], hi - lo, pub + 32UL*lo, sig + 64UL*lo, msg_off + lo, msg_sz + lo,
                                      blob, blob_sz, err + lo );
  } );
}

extern "C" int
fd_ed25519_amd_multi_verify_txns( fd_ed25519_amd_multi_t * m, ulong txn_cnt, uchar const * payload, uint const * txn_off,
                                  uint const * txn_sz, ulong payload_sz, schar * txn_err, uint * sig_base,
                                  schar * sig_err ) {
  if( !m || (txn_cnt && (!payload || !txn_off || !txn_sz || !txn_err)) ) return FD_ED25519_AMD_ERR_INVAL;
  if( sig_err && !sig_base ) return FD_ED25519_AMD_ERR_INVAL;
  fd_ed25519_amd_t const * e0 = m->eng[0];
  for( ulong t=0; t<txn_cnt; t++ ) {
    if( txn_sz[t] > FD_TXN_AMD_MTU || (ulong)txn_off[t] + txn_sz[t] > payload_sz || txn_sz[t] > e0->blob_cap )
      return FD_ED25519_AMD_ERR_INVAL;
    if( fd_amd_txn_slots1( payload + txn_off[t], txn_sz[t] ) > e0->cap ) return FD_ED25519_AMD_ERR_INVAL;
  }
  if( sig_base ) fd_ed25519_amd_txn_slots( txn_cnt, payload, txn_off, txn_sz, sig_base );   /* global numbering */
  if( !txn_cnt ) return FD_ED25519_AMD_OK;
  return run_all( m, [&]( ulong r ) -> int {
    ulong lo, hi;
    fd_ed25519_amd_shard_range( txn_cnt, m->ndev, r, &lo, &hi );
    if( lo == hi ) return FD_ED25519_AMD_OK;
    std::vector<uint> base( sig_base ? hi - lo + 1UL : 0UL );
    return fd_ed25519_amd_verify_txns( m->eng[r], hi - lo, payload, txn_off + lo, txn_sz + lo, payload_sz, txn_err + lo,
                                       sig_base ? base.data() : NULL, sig_err ? sig_err + sig_base[lo] : NULL );
  } );
}
