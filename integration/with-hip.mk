# config/extra/with-hip.mk -- build-side plug of the gfx950 ed25519 engine
# into the reference (anoushk1234/firedancer), modelled on
# config/extra/with-wd-f1.mk.  A maintainer copies this file to
# config/extra/ and builds with EXTRAS="hip" FD_HIP_ENGINE=<this repo>.
#
# Effect: -DFD_HAS_HIP=1 selects the wrap in src/ballet/ed25519/
# fd_ed25519_user.c (integration/fd_ed25519_user_hip.patch): the reference
# definitions of fd_ed25519_verify, fd_ed25519_verify_batch_single_msg and
# fd_ed25519_strerror compile out and the linker takes them from
# libfd_ed25519_hip.so, whose prototypes are the reference's
# (tests/test_ref_boundary.py compiles the reference header next to
# include/fd_ed25519_hip.h and links a fd_txn_verify-shaped caller).

FD_HIP_ENGINE ?= $(abspath ../firedancer_amd_engine)

CPPFLAGS += -DFD_HAS_HIP=1 -I$(FD_HIP_ENGINE)/include
LDFLAGS  += -L$(FD_HIP_ENGINE)/firedancer_amd -lfd_ed25519_hip \
            -Wl,-rpath,$(FD_HIP_ENGINE)/firedancer_amd -Wl,-rpath-link,/opt/rocm/lib
