extern "C" const char* ptts_build_id(void) { return "41ee0f1ab44425bc+probes"; }
