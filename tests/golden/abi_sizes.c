/* prints sizeof of every ABI struct; used by tests/test_abi.py */
#include <stdio.h>
#include <stddef.h>
#include "ksim_engine.h"
#include "ksim_trace.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n",sizeof(ksim_node),sizeof(ksim_pod),sizeof(ksim_typical),sizeof(ksim_result),sizeof(ksim_config),sizeof(ksim_trace_node),sizeof(ksim_trace_pod),sizeof(ksim_typical_cfg),sizeof(ksim_replay_cfg),sizeof(ksim_report),sizeof(ksim_power_report),sizeof(ksim_power_model));}
