# round 5: Nussbaumer with the two waves of a pair on one SIMD (512-thread
# workgroups of four pairs, waves p and p + 4; LDS sequence-number pair sync
# instead of the workgroup barrier), 16 or 1 units per pair, against the
# committed build
bash tools/gpu_session.sh abnus abnusref
