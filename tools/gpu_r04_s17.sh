#!/bin/bash
# Round-4 session: the bench's multi-rank path rehearsed with 2 ranks on the one GPU (gloo; the
# per-x cut alphas must equal N = 1's), and the distributed-refresh GPU tests
bash tools/gpu_session.sh gpurun_out/s17 \
  "rehearse|600|bash tools/rehearse_n2.sh 200000"
