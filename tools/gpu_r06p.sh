#!/bin/bash
# Round-6 session p: acff_persist NF 3 (96-row stages): classifier / int8 tests, classifier
# stage A/B against ab/head.so (b64, b8), bench A/B b64.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=r06p OLD=ab/head.so TESTS="tests/test_gpu_parity.py tests/test_gpu_int8.py tests/test_gpu_pipeline.py tests/test_cli.py" KEXPR="classifier or acff or redconv or int8 or two_stage or cli or batch_edges" CLS="64 8" BENCHES="--batch 64" bash tools/ab_session.sh
