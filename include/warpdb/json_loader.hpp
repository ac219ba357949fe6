// json_loader.hpp -- line-delimited {"price": .., "quantity": ..} records
// (reference include/json_loader.hpp, src/json_loader.cpp:16-53).
#pragma once
#include "csv_loader.hpp"

HostTable load_json_to_host(const std::string &filepath);
Table load_json_to_gpu(const std::string &filepath, int device = 0);
