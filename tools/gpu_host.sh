# Host-resident paths: API tests + PCIe-inclusive timings (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/host; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_warpdb_api.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 ./tools/pcie_bench > $O/pcie_bench.txt 2>&1
for C in 8388608 33554432 134217728; do
  echo "== chunk $C" >> $O/pcie_chunks.txt
  WARPDB_HOST_CHUNK_ROWS=$C timeout -k 10 300 ./tools/pcie_bench >> $O/pcie_chunks.txt 2>&1
done
echo ok
