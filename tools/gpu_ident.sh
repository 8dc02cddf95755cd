# Two-build check: bit identity of every output (old = ab_old/ build, new =
# in-tree), then interleaved benches of both (tools/gpu_libab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
SAMNERF_LIB="$GRAFT_REPO_ROOT/ab_old/libsamnerf_hip.so" timeout -k 10 200 python tools/diag/build_identity.py "$OUT/id_old.npz" > "$OUT/id_old.log" 2>&1 || { tail -5 "$OUT/id_old.log"; exit 1; }
timeout -k 10 200 python tools/diag/build_identity.py "$OUT/id_new.npz" > "$OUT/id_new.log" 2>&1 || { tail -5 "$OUT/id_new.log"; exit 1; }
python tools/diag/build_identity.py compare "$OUT/id_old.npz" "$OUT/id_new.npz"
rm -f "$OUT/id_old.npz" "$OUT/id_new.npz"
bash tools/gpu_libab.sh
