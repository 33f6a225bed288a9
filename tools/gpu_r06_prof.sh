#!/bin/bash
# Round-6 profile session: the driver's command (storm) and the ssn |V| = 16384 config under
# rocprofv3 -- a kernel trace and five separate PMC passes each (tools/profile_r06.sh).
set -u
bash tools/profile_r06.sh r06storm || exit 1
bash tools/profile_r06.sh r06ssn --instance ssn --scenarios 100000 --vertices 16384 || exit 1
