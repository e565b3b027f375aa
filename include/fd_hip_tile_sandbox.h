#ifndef HEADER_fd_hip_tile_sandbox_h
#define HEADER_fd_hip_tile_sandbox_h

/* fd_hip_tile_sandbox.h -- what a reference tile that drives the engine
   needs to keep through fd_sandbox (util/sandbox/fd_sandbox.c), shared by
   the patched verify tile (integration/fd_verify_tile_hip.patch) and replay
   tile (integration/fd_replay_hip.patch).  Header-only, plain C.

   fd_hip_tile_device_fds: the descriptors the HIP runtime opened in
   privileged_init (/dev/kfd, /dev/dri/...), for populate_allowed_fds and the
   ioctl rule below.

   fd_hip_tile_seccomp: the tile's reference policy (fd_verify_tile and
   fd_replay_tile .seccomppolicy: write to stderr or the logfile, fsync the
   logfile) plus what the HIP runtime does on the tile's thread, arguments
   checked where a call could widen the sandbox:
     ioctl                    only on the device fds above (queue and event
                              management)
     mmap, mprotect           never with PROT_EXEC (host allocations its
                              internal pools grow under load)
     munmap, madvise, mbind,
     get_mempolicy            (those allocations and their NUMA placement)
     futex, sched_yield       its locks
     clock_nanosleep, nanosleep, getpid, gettid, sched_getaffinity,
     rt_sigreturn, exit, exit_group
   The list was measured: tests/test_gpu_tile_hip.py runs the patched verify
   tile under this filter with SECCOMP_RET_TRAP as fail_action and requires
   zero traps.  The runtime's own threads, started in privileged_init, are
   not under the tile thread's filter, and a process with threads cannot
   enter fd_sandbox's user namespace: the tiles run with the sandbox
   disabled. */

#include <dirent.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <linux/audit.h>
#include <linux/filter.h>
#include <linux/seccomp.h>
#include <sys/mman.h>
#include <sys/syscall.h>

#define FD_HIP_TILE_FD_MAX (16UL)

/* Fills fd[0,max) with the HIP device descriptors open in this process.
   Returns the count, or -1 if /proc/self/fd is unreadable or there are
   more than max. */
static inline long
fd_hip_tile_device_fds( int * fd, unsigned long max ) {
  long cnt = 0L;
  DIR * dir = opendir( "/proc/self/fd" );
  if( !dir ) return -1L;
  for( struct dirent * e; (e = readdir( dir )); ) {
    char path[ 64 ], target[ 64 ];
    if( e->d_name[0]=='.' ) continue;
    int d = atoi( e->d_name );
    if( d==dirfd( dir ) ) continue;
    snprintf( path, sizeof(path), "/proc/self/fd/%d", d );
    long len = (long)readlink( path, target, sizeof(target)-1UL );
    if( len<=0L ) continue;
    target[ len ] = '\0';
    if( strncmp( target, "/dev/kfd", 8UL ) && strncmp( target, "/dev/dri/", 9UL ) ) continue;
    if( (unsigned long)cnt>=max ) { cnt = -1L; break; }
    fd[ cnt++ ] = d;
  }
  closedir( dir );
  return cnt;
}

/* Writes the filter into out[0,out_cnt).  Returns its instruction count,
   or 0 if out_cnt is too small or fd_cnt > FD_HIP_TILE_FD_MAX. */
static inline unsigned long
fd_hip_tile_seccomp( unsigned long        out_cnt,
                     struct sock_filter * out,
                     unsigned int         logfile_fd,
                     int const *          fd,
                     unsigned long        fd_cnt,
                     unsigned int         fail_action ) {
  static long const any[] = { SYS_munmap, SYS_madvise, SYS_futex, SYS_sched_yield, SYS_clock_nanosleep,
                              SYS_nanosleep, SYS_getpid, SYS_gettid, SYS_rt_sigreturn, SYS_exit, SYS_exit_group,
                              SYS_get_mempolicy, SYS_mbind, SYS_sched_getaffinity };
  unsigned long const nany = sizeof(any)/sizeof(any[0]);
  /* instruction indices of the blocks */
  unsigned long const i_fds   = 6UL;                                  /* ioctl: one JEQ per device fd */
  unsigned long const i_nr    = i_fds + fd_cnt + 1UL;                 /* the other calls by number */
  unsigned long const i_prot  = i_nr + 1UL + 2UL + nany + 2UL + 1UL;  /* mmap / mprotect: PROT_EXEC? */
  unsigned long const i_write = i_prot + 4UL;                         /* write: stderr or the logfile */
  unsigned long const i_fsync = i_write + 4UL;                        /* fsync: the logfile */
  unsigned long const i_allow = i_fsync + 3UL;
  unsigned long const cnt     = i_allow + 1UL;
  if( out_cnt<cnt || fd_cnt>FD_HIP_TILE_FD_MAX ) return 0UL;
  unsigned long i = 0UL;
#define TO( at ) ((unsigned char)((at) - i - 1UL))
#define STMT( c, k )        out[ i ] = (struct sock_filter)BPF_STMT( (c), (k) ), i++
#define JUMP( c, k, t, f )  out[ i ] = (struct sock_filter)BPF_JUMP( (c), (k), (t), (f) ), i++
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, arch ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, AUDIT_ARCH_X86_64, 1, 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, nr ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_ioctl, 0, TO( i_nr ) );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[0] ) );
  for( unsigned long k=0UL; k<fd_cnt; k++ ) JUMP( BPF_JMP | BPF_JEQ | BPF_K, (unsigned int)fd[ k ], TO( i_allow ), 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, nr ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_mmap,     TO( i_prot ), 0 );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_mprotect, TO( i_prot ), 0 );
  for( unsigned long k=0UL; k<nany; k++ ) JUMP( BPF_JMP | BPF_JEQ | BPF_K, (unsigned int)any[ k ], TO( i_allow ), 0 );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_write, TO( i_write ), 0 );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_fsync, TO( i_fsync ), 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[2] ) );
  JUMP( BPF_JMP | BPF_JSET | BPF_K, PROT_EXEC, 0, 1 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_RET | BPF_K, SECCOMP_RET_ALLOW );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[0] ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, 2, TO( i_allow ), 0 );                     /* stderr */
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, logfile_fd, TO( i_allow ), 0 );            /* the logfile */
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[0] ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, logfile_fd, TO( i_allow ), 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_RET | BPF_K, SECCOMP_RET_ALLOW );
#undef JUMP
#undef STMT
#undef TO
  return i==cnt ? cnt : 0UL;
}

#endif /* HEADER_fd_hip_tile_sandbox_h */
