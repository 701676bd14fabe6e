/* firedancer_amd/csrc/fd_numa.cpp
 *
 * NUMA placement of the host side of a GPU engine.  The reference pins
 * every tile to a core (src/app/frank/fd_frank_main.c:118-143) and lays the
 * tiles out so each verify tile's input link is local to it
 * (src/app/frank/fd_frank_init:67-80).  The host side of an engine here is
 * its pinned staging (written by the host thread, read by the GPU's DMA)
 * and the thread that stages: both belong on the NUMA node the GPU hangs
 * off.  The node comes from sysfs:
 *
 *   hipDeviceGetPCIBusId -> <root>/bus/pci/devices/<bdf>/numa_node
 *                        -> <root>/devices/system/node/node<N>/cpulist
 *
 * fd_ed25519_amd_sysfs_numa reads an arbitrary sysfs root, so the parsing
 * is tested on a synthetic tree (tests/test_numa.py).
 */
#include <hip/hip_runtime.h>
#include <ctype.h>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/fd_ed25519_amd.h"
#include "fd_ed25519_engine.h"

#define MPOL_DEFAULT_   (0)
#define MPOL_PREFERRED_ (1)
#define NODE_WORDS      (16)   /* up to 1024 NUMA nodes */

static int
read_small( char const * path, char * buf, ulong sz ) {
  FILE * f = fopen( path, "r" );
  if( !f ) return -1;
  ulong n = fread( buf, 1, sz - 1UL, f );
  fclose( f );
  buf[n] = '\0';
  return (int)n;
}

/* "0-3,8,10-11\n" -> cpus[] (at most cpus_max); returns the count, -1 on a
   malformed list */
static int
parse_cpulist( char const * s, int * cpus, int cpus_max ) {
  int cnt = 0;
  while( *s && *s != '\n' ) {
    if( !isdigit( (uchar)*s ) ) return -1;
    char * e; long a = strtol( s, &e, 10 ), b = a;
    if( *e == '-' ) { b = strtol( e + 1, &e, 10 ); if( b < a ) return -1; }
    for( long c = a; c <= b; c++ ) { if( cnt < cpus_max ) cpus[cnt] = (int)c; cnt++; }
    s = e;
    if( *s == ',' ) s++;
    else if( *s && *s != '\n' ) return -1;
  }
  return cnt < cpus_max ? cnt : cpus_max;
}

extern "C" int
fd_ed25519_amd_sysfs_numa( char const * sysfs_root, char const * pci_bdf, int * node, int * cpus, int cpus_max ) {
  if( !sysfs_root || !pci_bdf || !node || (cpus_max > 0 && !cpus) ) return -1;
  char bdf[64]; ulong k = 0;
  for( ; pci_bdf[k] && k < sizeof(bdf) - 1UL; k++ ) bdf[k] = (char)tolower( (uchar)pci_bdf[k] );
  bdf[k] = '\0';
  char path[512], buf[4096];
  snprintf( path, sizeof path, "%s/bus/pci/devices/%s/numa_node", sysfs_root, bdf );
  *node = -1;
  if( read_small( path, buf, sizeof buf ) <= 0 ) return -1;
  int nd = atoi( buf );
  if( nd < 0 ) return 0;                           /* the platform reports no node */
  *node = nd;
  if( cpus_max <= 0 ) return 0;
  snprintf( path, sizeof path, "%s/devices/system/node/node%d/cpulist", sysfs_root, nd );
  if( read_small( path, buf, sizeof buf ) < 0 ) return -1;
  return parse_cpulist( buf, cpus, cpus_max );
}

extern "C" int
fd_ed25519_amd_device_numa_node( int device ) {
  char bdf[64];
  if( hipDeviceGetPCIBusId( bdf, (int)sizeof bdf, device ) != hipSuccess ) { (void)hipGetLastError(); return -1; }
  int node = -1;
  (void)fd_ed25519_amd_sysfs_numa( "/sys", bdf, &node, NULL, 0 );
  return node;
}

/* Bind the calling thread to `device`'s NUMA node: its CPUs (those of them
   the thread may use; unchanged if none) and, for memory, the node as the
   preferred one.  Returns the node, or -1 when the node is unknown.  With
   FD_ED25519_AMD_NUMA=0 nothing is changed. */
int
fd_amd_numa_bind_thread( int device ) {
  char const * env = getenv( "FD_ED25519_AMD_NUMA" );
  if( env && !strcmp( env, "0" ) ) return -1;
  char bdf[64];
  if( hipDeviceGetPCIBusId( bdf, (int)sizeof bdf, device ) != hipSuccess ) { (void)hipGetLastError(); return -1; }
  static int cpus[4096];
  static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  pthread_mutex_lock( &mu );
  int node = -1, n = fd_ed25519_amd_sysfs_numa( "/sys", bdf, &node, cpus, 4096 );
  cpu_set_t allowed, want; CPU_ZERO( &want );
  int hits = 0;
  if( node >= 0 && n > 0 && !sched_getaffinity( 0, sizeof allowed, &allowed ) ) {
    for( int i=0; i<n; i++ ) if( cpus[i] < CPU_SETSIZE && CPU_ISSET( cpus[i], &allowed ) ) { CPU_SET( cpus[i], &want ); hits++; }
  }
  pthread_mutex_unlock( &mu );
  if( node < 0 ) return -1;
  if( hits ) (void)pthread_setaffinity_np( pthread_self(), sizeof want, &want );
  unsigned long mask[NODE_WORDS]; memset( mask, 0, sizeof mask );
  if( node < 64 * NODE_WORDS ) {
    mask[node / 64] |= 1UL << (node % 64);
    (void)syscall( SYS_set_mempolicy, MPOL_PREFERRED_, mask, (unsigned long)(64 * NODE_WORDS + 1) );
  }
  return node;
}

/* Allocation-only form for engines created on a caller's thread: prefer the
   device's node while the engine's pinned staging is allocated, then put
   the thread's policy back (the caller's affinity is never touched). */
int
fd_amd_numa_prefer_begin( int device, int * saved_mode, unsigned long * saved_mask /* NODE_WORDS */ ) {
  char const * env = getenv( "FD_ED25519_AMD_NUMA" );
  if( env && !strcmp( env, "0" ) ) return -1;
  int node = fd_ed25519_amd_device_numa_node( device );
  if( node < 0 || node >= 64 * NODE_WORDS ) return -1;
  memset( saved_mask, 0, sizeof(unsigned long) * NODE_WORDS );
  if( syscall( SYS_get_mempolicy, saved_mode, saved_mask, (unsigned long)(64 * NODE_WORDS + 1), NULL, 0UL ) ) return -1;
  unsigned long mask[NODE_WORDS]; memset( mask, 0, sizeof mask );
  mask[node / 64] |= 1UL << (node % 64);
  if( syscall( SYS_set_mempolicy, MPOL_PREFERRED_, mask, (unsigned long)(64 * NODE_WORDS + 1) ) ) return -1;
  return node;
}

void
fd_amd_numa_prefer_end( int saved_mode, unsigned long const * saved_mask ) {
  (void)syscall( SYS_set_mempolicy, saved_mode, saved_mode == MPOL_DEFAULT_ ? NULL : saved_mask,
                 saved_mode == MPOL_DEFAULT_ ? 0UL : (unsigned long)(64 * NODE_WORDS + 1) );
}
