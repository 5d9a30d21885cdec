# SQ counters of the default library and the lib_v0 variant (A/B), short bench runs
set -o pipefail
cd /root/repo
bash tools/sq_profile.sh v2 --no-extra --no-pipelined --steps 5 --warmup 2 && \
DCAMD_LIB=$PWD/data-compression_amd/lib_v0/libdcamd.so bash tools/sq_profile.sh v0 --no-extra --no-pipelined --steps 5 --warmup 2
