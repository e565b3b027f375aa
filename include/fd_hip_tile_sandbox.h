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
#include <errno.h>
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

/* ---- the GPU-owning process (service mode's GPU tile) -----------------------

   fd_hip_tile_seccomp_process: the filter for EVERY thread of the process
   that owns a HIP context (integration/svc_run.c, integration/
   fd_verify_gpu_tile.c), installed with SECCOMP_FILTER_FLAG_TSYNC: the
   calls above, plus what the HIP runtime's own threads and the service's
   teardown do (measured on MI355X: tests/test_gpu_svc_sandbox.py runs the
   service under this filter with SECCOMP_RET_TRAP and requires no trap):
     ioctl only on the device fds; mmap / mprotect never with PROT_EXEC;
     munmap, mremap, madvise, brk; futex, sched_yield, the sleeps and
     clocks; the signal-mask calls and rt_sigreturn; poll / ppoll and read
     (the runtime's event waits); getpid, gettid; exit, exit_group; write to
     stderr or the logfile, fsync the logfile.
   open / openat fail with EACCES rather than end the process: the HSA
   runtime reads /proc/self/maps and std::random_device opens /dev/random
   lazily after the sandbox is entered (measured: profiles/r06/sandbox.md)
   and both take a failed open.
   Not in it: socket, connect, clone / clone3 / fork /
   execve, ptrace, kill / tgkill (other processes), prctl, seccomp, mount,
   unshare -- the process cannot start a thread or program, reach a file,
   the network or another process. */
static inline unsigned long
fd_hip_tile_seccomp_process( unsigned long        out_cnt,
                             struct sock_filter * out,
                             unsigned int         logfile_fd,
                             int const *          fd,
                             unsigned long        fd_cnt,
                             unsigned int         fail_action ) {
  static long const any[] = { SYS_munmap, SYS_mremap, SYS_madvise, SYS_brk, SYS_futex, SYS_sched_yield,
                              SYS_clock_nanosleep, SYS_nanosleep, SYS_clock_gettime, SYS_clock_getres, SYS_gettimeofday,
                              SYS_getpid, SYS_gettid, SYS_rt_sigreturn, SYS_rt_sigprocmask, SYS_sigaltstack,
                              SYS_exit, SYS_exit_group, SYS_get_mempolicy, SYS_mbind, SYS_sched_getaffinity,
                              SYS_poll, SYS_ppoll, SYS_read, SYS_restart_syscall };
  unsigned long const nany = sizeof(any)/sizeof(any[0]);
  unsigned long const i_fds   = 6UL;
  unsigned long const i_nr    = i_fds + fd_cnt + 1UL;
  unsigned long const i_prot  = i_nr + 1UL + 2UL + nany + 4UL + 1UL;
  unsigned long const i_write = i_prot + 4UL;
  unsigned long const i_fsync = i_write + 4UL;
  unsigned long const i_deny  = i_fsync + 3UL;
  unsigned long const i_allow = i_deny + 1UL;
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
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_open,   TO( i_deny ), 0 );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, SYS_openat, TO( i_deny ), 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[2] ) );
  JUMP( BPF_JMP | BPF_JSET | BPF_K, PROT_EXEC, 0, 1 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_RET | BPF_K, SECCOMP_RET_ALLOW );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[0] ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, 2, TO( i_allow ), 0 );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, logfile_fd, TO( i_allow ), 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, args[0] ) );
  JUMP( BPF_JMP | BPF_JEQ | BPF_K, logfile_fd, TO( i_allow ), 0 );
  STMT( BPF_RET | BPF_K, fail_action );
  STMT( BPF_RET | BPF_K, SECCOMP_RET_ERRNO | (EACCES & SECCOMP_RET_DATA) );
  STMT( BPF_RET | BPF_K, SECCOMP_RET_ALLOW );
#undef JUMP
#undef STMT
#undef TO
  return i==cnt ? cnt : 0UL;
}

/* fd_hip_tile_sandbox_process: what fd_sandbox_enter
   (src/util/sandbox/fd_sandbox.c:573-719, entered from fd_topo_run.c:122)
   does that a process with threads can take.  Its user namespace and
   pivot_root need one thread (unshare( CLONE_NEWUSER ) refuses a threaded
   process, fd_sandbox.c:649) and the HIP runtime has started its own; the
   rest applies to the whole process:
     1. the descriptors: every open fd is stderr, the logfile (logfile_fd,
        -1: none), a HIP device fd (/dev/kfd, /dev/dri/...), an anonymous
        inode of the runtime's or the launcher's pipe; any other is an error, as
        fd_sandbox_private_check_exact_file_descriptors makes it
     2. rlimits (fd_sandbox_private_set_rlimits): NOFILE at the highest open
        fd + 1, NPROC 0 (no new process or thread), CORE, NICE, MSGQUEUE,
        RTPRIO, RTTIME 0 (AS, DATA, STACK and MEMLOCK stay: the runtime maps
        and pins the GPU's address space)
     3. capabilities (fd_sandbox_private_drop_caps): the bounding set dropped
        and the securebits locked where CAP_SETPCAP allows; none permitted,
        effective, inheritable or ambient
     4. PR_SET_NO_NEW_PRIVS, PR_SET_DUMPABLE as asked
     5. fd_hip_tile_seccomp_process over every thread (SECCOMP_FILTER_FLAG_TSYNC)
   The caller has switched uid and gid already (fd_topo_run.c does it for a
   tile that skips fd_sandbox_enter).  Returns 0, or -1 with the step that
   failed in why[0,why_sz). */
#include <errno.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <linux/capability.h>
#include <linux/securebits.h>

#ifndef SECCOMP_FILTER_FLAG_TSYNC
#define SECCOMP_FILTER_FLAG_TSYNC (1UL)
#endif

static inline int
fd_hip_tile_sandbox_process( int            logfile_fd,
                             int const *    dev_fd,
                             unsigned long  dev_cnt,
                             int            dumpable,
                             unsigned int   fail_action,
                             char *         why,
                             unsigned long  why_sz ) {
#define FAIL( ... ) do { snprintf( why, why_sz, __VA_ARGS__ ); return -1; } while( 0 )
  /* 1. descriptors */
  int hi = 2;
  {
    DIR * dir = opendir( "/proc/self/fd" );
    if( !dir ) FAIL( "opendir(/proc/self/fd) failed (%d)", errno );
    int bad = -1; char bad_target[ 96 ] = { 0 };
    for( struct dirent * e; (e = readdir( dir )); ) {
      if( e->d_name[0]=='.' ) continue;
      int d = atoi( e->d_name );
      if( d==dirfd( dir ) ) continue;
      char path[ 64 ], target[ 96 ];
      snprintf( path, sizeof(path), "/proc/self/fd/%d", d );
      long len = (long)readlink( path, target, sizeof(target)-1UL );
      if( len<=0L ) continue;
      target[ len ] = '\0';
      /* anonymous inodes are the runtime's (events, dma-bufs); a pipe is the
         launcher's (fd_topo_run's allow_fd, the parent's death watch) */
      int ok = d==2 || d==logfile_fd || !strncmp( target, "anon_inode:", 11UL ) || !strncmp( target, "pipe:", 5UL );
      for( unsigned long k=0UL; k<dev_cnt; k++ ) ok |= d==dev_fd[ k ];
      if( !ok && bad<0 ) { bad = d; snprintf( bad_target, sizeof(bad_target), "%s", target ); }
      if( d>hi ) hi = d;
    }
    closedir( dir );
    if( bad>=0 ) FAIL( "fd %d (%s) is not stderr, the logfile or a HIP device", bad, bad_target );
  }
  /* 2. rlimits */
  {
    struct { int res; unsigned long lim; } rl[] = {
      { RLIMIT_NOFILE, (unsigned long)hi + 1UL }, { RLIMIT_NPROC, 0UL }, { RLIMIT_CORE, 0UL }, { RLIMIT_NICE, 0UL },
      { RLIMIT_MSGQUEUE, 0UL }, { RLIMIT_RTPRIO, 0UL }, { RLIMIT_RTTIME, 0UL } };
    for( unsigned long k=0UL; k<sizeof(rl)/sizeof(rl[0]); k++ ) {
      if( dumpable && rl[ k ].res==RLIMIT_CORE ) continue;
      struct rlimit l = { rl[ k ].lim, rl[ k ].lim };
      if( setrlimit( rl[ k ].res, &l ) ) FAIL( "setrlimit(%d, %lu) failed (%d)", rl[ k ].res, rl[ k ].lim, errno );
    }
  }
  /* 3. capabilities */
  {
    struct __user_cap_header_struct hdr = { _LINUX_CAPABILITY_VERSION_3, 0 };
    struct __user_cap_data_struct   cap[ 2 ];
    memset( cap, 0, sizeof(cap) );
    if( syscall( SYS_capget, &hdr, cap ) ) FAIL( "capget failed (%d)", errno );
    if( cap[ CAP_TO_INDEX( CAP_SETPCAP ) ].effective & CAP_TO_MASK( CAP_SETPCAP ) ) {
      if( prctl( PR_SET_SECUREBITS, SECBIT_KEEP_CAPS_LOCKED | SECBIT_NO_SETUID_FIXUP | SECBIT_NO_SETUID_FIXUP_LOCKED |
                 SECBIT_NOROOT | SECBIT_NOROOT_LOCKED | SECBIT_NO_CAP_AMBIENT_RAISE | SECBIT_NO_CAP_AMBIENT_RAISE_LOCKED ) )
        FAIL( "prctl(PR_SET_SECUREBITS) failed (%d)", errno );
      for( unsigned long c=0UL; c<=63UL; c++ ) if( prctl( PR_CAPBSET_DROP, c, 0, 0, 0 ) && errno!=EINVAL )
        FAIL( "prctl(PR_CAPBSET_DROP, %lu) failed (%d)", c, errno );
    }
    memset( cap, 0, sizeof(cap) );
    if( syscall( SYS_capset, &hdr, cap ) ) FAIL( "capset failed (%d)", errno );
    if( prctl( PR_CAP_AMBIENT, PR_CAP_AMBIENT_CLEAR_ALL, 0, 0, 0 ) ) FAIL( "prctl(PR_CAP_AMBIENT_CLEAR_ALL) failed (%d)", errno );
  }
  /* 4. */
  if( prctl( PR_SET_DUMPABLE, dumpable ) ) FAIL( "prctl(PR_SET_DUMPABLE) failed (%d)", errno );
  if( prctl( PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0 ) ) FAIL( "prctl(PR_SET_NO_NEW_PRIVS) failed (%d)", errno );
  /* 5. every thread */
  struct sock_filter filter[ 128 ];
  unsigned long n = fd_hip_tile_seccomp_process( 128UL, filter, logfile_fd>=0 ? (unsigned int)logfile_fd : 2U, dev_fd, dev_cnt,
                                                 fail_action );
  if( !n ) FAIL( "seccomp filter does not fit (%lu device fds)", dev_cnt );
  struct sock_fprog prog = { (unsigned short)n, filter };
  long r = syscall( SYS_seccomp, SECCOMP_SET_MODE_FILTER, SECCOMP_FILTER_FLAG_TSYNC, &prog );
  if( r ) FAIL( "seccomp(TSYNC) failed (%ld, errno %d)", r, errno );
#undef FAIL
  return 0;
}

#endif /* HEADER_fd_hip_tile_sandbox_h */
