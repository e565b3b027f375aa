# config/extra/with-hip.mk -- build-side plug of the gfx950 ed25519 engine
# into the reference (anoushk1234/firedancer), modelled on
# config/extra/with-wd-f1.mk.  A maintainer copies this file to
# config/extra/ and builds with EXTRAS="hip" FD_HIP_ENGINE=<this repo>.
#
# Two link modes (FD_HIP_PLUG):
#
#   selective (default, recommended)
#       -DFD_HAS_HIP=1 turns on the GPU batch paths of the patched tiles
#       (integration/fd_verify_tile_hip.patch, fd_replay_hip.patch), which
#       call the engine's batch entry points (fd_verify_hip_tile_*,
#       fd_replay_hip_*).  fd_ed25519_verify and
#       fd_ed25519_verify_batch_single_msg stay the reference's CPU code, so
#       the latency-bound callers -- TLS (src/waltz/tls/fd_tls.c:907), gossip
#       vote verify, the FEC resolver (src/disco/shred/fd_fec_resolver.c:476),
#       the ed25519 precompile -- keep a host core's ~15 us per call instead
#       of a lone GPU call's ~300 us.
#
#   full
#       additionally -DFD_HAS_HIP_DROPIN=1, which selects the wrap in
#       src/ballet/ed25519/fd_ed25519_user.c
#       (integration/fd_ed25519_user_hip.patch): the reference definitions of
#       fd_ed25519_verify, fd_ed25519_verify_batch_single_msg and
#       fd_ed25519_strerror compile out and the linker takes them from
#       libfd_ed25519_hip.so, whose prototypes are the reference's -- every
#       caller goes to the GPU through the drop-in.
#
# tests/test_ref_boundary.py builds and checks both modes.

FD_HIP_ENGINE ?= $(abspath ../firedancer_amd_engine)
FD_HIP_PLUG   ?= selective

CPPFLAGS += -DFD_HAS_HIP=1 -I$(FD_HIP_ENGINE)/include
ifeq ($(FD_HIP_PLUG),full)
CPPFLAGS += -DFD_HAS_HIP_DROPIN=1
else ifneq ($(FD_HIP_PLUG),selective)
$(error FD_HIP_PLUG must be selective or full)
endif
LDFLAGS  += -L$(FD_HIP_ENGINE)/firedancer_amd -lfd_ed25519_hip \
            -Wl,-rpath,$(FD_HIP_ENGINE)/firedancer_amd -Wl,-rpath-link,/opt/rocm/lib
