#!/bin/bash
# Round-6 session ze: the fused classifier front's stem stores as buffer stores: classifier
# tests, per-stage classifier times against ab/head.so.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=r06ze OLD=ab/head.so TESTS="tests/test_gpu_stem.py tests/test_gpu_parity.py" KEXPR="front or classifier or stem or cli" CLS="64 8" bash tools/ab_session.sh || exit $?
