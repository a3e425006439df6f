source tools/../run_gpu_steps.sh
cd "$GRAFT_REPO_ROOT"
export EEGAN_GTERM_GRAD_EARLY=-1
step 400 early_tests python3 -u -m pytest tests/test_gpu_models.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread -k "full_step or graph_matches or adam"
unset EEGAN_GTERM_GRAD_EARLY
SETTINGS="base EEGAN_GTERM_GRAD_EARLY=2 EEGAN_GTERM_GRAD_EARLY=-1" ROUNDS=2 bash tools/gpu_env_ab.sh
