#!/bin/bash
# round 6 closing evidence, part 2: rocprofv3 passes (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ)
# of cfg2 (the default line's workload), cfg1, cfg3 and cfg4
cd "$GRAFT_REPO_ROOT"
tools/evidence.sh cfg2 cfg1 cfg3 cfg4
