// orbfe_lib.hip — single translation unit of liborbfe.so (kernels, their launches and the
// __constant__ tables they read must share one code object).
#include "orbfe_extract.hip"
#include "orbfe_stereo.hip"
#include "orbfe_api.hip"
#include "orbfe_match.hip"
#include "orbfe_greedy.hip"
#include "orbfe_match_api.hip"
#include "orbfe_bow.hip"
#include "orbfe_archive.hip"
