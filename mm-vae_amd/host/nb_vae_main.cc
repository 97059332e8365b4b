// Drop-in for src/nb_vae_main.cc: Negative-Binomial VAE training on the MI355X engine.
#include "cli.hh"

int main(int argc, const char* argv[]) { return mmvae_host::run_cli(argc, argv, MMVAE_MODEL_NB); }
