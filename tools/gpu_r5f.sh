# round 5: Nussbaumer without SGPR spills (prefetch only at M32 n=2048; the
# final barrier skip compile-time) and LDS padded to 40 KiB at n <= 1024 (4
# workgroups per CU), against the committed build; then the Nussbaumer tests
bash tools/gpu_session.sh abnus abnusref nustest
