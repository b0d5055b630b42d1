set -o pipefail
mkdir -p gpurun_out/t2
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_invariant.py "tests/test_gpu_xgmi.py::test_xgmi_engine_tp_f32_model_matches_single_exactly" "tests/test_gpu_xgmi.py::test_api_on_gpu_concurrent_equals_solo" "tests/test_gpu_xgmi.py::test_data_plane_bytes_reported" "tests/test_gpu_xgmi.py::test_xgmi_engine_tp_matches_single" "tests/test_gpu_engine.py::test_compute_only_rank_fused_matches_separate" "tests/test_gpu_engine.py::test_attn_block_matches_separate_kernels" > gpurun_out/t2/pytest.log 2>&1
