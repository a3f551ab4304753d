// jmh_flow.hip — k_mb_flow, the dataflow wavefront: jmh_analyse.hip's device
// functions (me_mb, intra_role, the intra decisions) with jmh_final.h's final_core, in a
// translation unit of their own so that the tick kernels' register allocation stays as it was.
#define JMH_FLOW_TU 1
#include "jmh_analyse.hip"
