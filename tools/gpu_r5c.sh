# round 5: n = 8192 transforms at 12 waves (3 per SIMD) with the register
# stages pinned apart (BIG_PIN) and the first polynomial loaded after the
# table prologue (BIG_LATE_LOAD), vs the product build; n = 4096 with the pins
bash tools/gpu_session.sh abl_8192 abl_4096
