// Drop-in for src/vmf_vae_main.cc: von Mises-Fisher VAE training on the MI355X engine.
#include "cli.hh"

int main(int argc, const char* argv[]) { return mmvae_host::run_cli(argc, argv, MMVAE_MODEL_VMF); }
