"""Diffusion models: SD3 MMDiT, VAE, CLIP / T5 text encoders, samplers and the SD3 pipeline."""
