# round 5: Nussbaumer with this wave's own block results read before the
# results barrier (NUS_PREREAD) against the product build
bash tools/gpu_session.sh abnus
