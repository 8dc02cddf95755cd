set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r6v STEPS="tests" PYTEST_ARGS="-s" PYTEST_FILES="tests/test_gpu_pdf_split.py" bash tools/gpu_run.sh
