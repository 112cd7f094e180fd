# A/B: speculative round trip, variant A (shared registers): slower, see profiles/r02_encoder_ab_specrt.txt
