# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/copy_probe:
# every variant moves 512 MiB of reads and a known write count per launch),
# for the access kinds the stage uses: 16-B/lane plain and nontemporal loads,
# plain and nontemporal stores.  MI355X_MICROARCH.md: calibrate on your own
# access pattern before trusting an absolute.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/fetch_calib
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- ./tools/copy_probe > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- ./tools/copy_probe > $OUT/write.log 2>&1 || exit 2
