# round 3: the new parity tests (full-size lane layout, slicer near-ties,
# flagged batches, scratch-grow failure, any first) and the FSK live-column layout
set -o pipefail
T=${T:-r3a}
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fsk.py tests/test_gpu_slicer.py \
  "tests/test_gpu_parity.py::test_full_size_lane_layout_as_benched" \
  "tests/test_gpu_parity.py::test_fec_fused_after_8psk_demod" \
  "tests/test_gpu_parity.py::test_batch_of_flagged_streams" \
  "tests/test_gpu_parity.py::test_failed_scratch_grow_leaves_plan_usable" \
  "tests/test_gpu_parity.py::test_lane_layout_any_first" \
  "tests/test_gpu_parity.py::test_exact_complex_lowpass_path_matches" \
  "tests/test_gpu_parity.py::test_silence_cases_take_exact_path" \
  -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; exit $rc
