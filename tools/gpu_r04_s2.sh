#!/bin/bash
# Round-4 profile session: the driver's command under rocprofv3 (trace + PMC passes)
bash tools/gpu_session.sh gpurun_out/s3 "profile|1100|bash tools/profile_r04.sh r04"
