# GPU parity for the deferred gather pass, then same-box A/B (PM_GATHER_DEFER) on C2, C3, C5
set -u
O=gpurun_out/dfr; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "gather or full or scene_parity or render or c5 or sharded or reset or pbrt" > $O/pytest.log 2>&1 || exit $?
for c in c2 c3 c5; do CFG=$c QTAG=dfr bash tools/envcmp.sh PM_GATHER_DEFER=1 PM_GATHER_DEFER=0 || exit $?; done
