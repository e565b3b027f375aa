#!/bin/bash
tools/r05i_session.sh || exit $?
tools/r05j_session.sh
