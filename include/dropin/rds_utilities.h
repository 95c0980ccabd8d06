// rds_utilities.h (drop-in) -- RDS symbol/bit recovery and frame layer of the reference
// (include/rds_utilities.h:6-19). cdr/manchester/differential run on the MI355X kernels; the
// serial frame sync and group parser (start_frame_sync, check_block, parse) run on the host.
#ifndef SDR_DROPIN_RDS_UTILITIES_H
#define SDR_DROPIN_RDS_UTILITIES_H

#include <algorithm>
#include <cstdint>
#include <deque>
#include <iostream>
#include <string>
#include <vector>

int cdr(int sps, const std::vector<float> &signal);
void manchester_decode(std::vector<int> &bits, const std::vector<int> &symbols, int &block_count, int &half_symbol,
                       int &start);
void differential_decode(std::vector<int> &decoded_bits, const std::vector<int> &bits, int &last_bit, int &block_num);
void parse(const uint64_t &bytes, uint64_t &chars, uint64_t &output, bool &first_time);
void check_block(std::string &offset_type, std::vector<int>::iterator bitstream_start,
                 std::vector<int>::iterator bitstream_end, uint64_t &reg, uint64_t &chars, uint64_t &output,
                 bool &first_time, std::deque<std::string> &window);
// rds_utilities.h:16 -- the reference's alternative bit-serial synchroniser (never called by its
// program; served for API completeness, host/rds_frame.cpp)
void error_detection(uint64_t &reg, uint64_t &chars, uint64_t &output, bool &first_time, int &sync, int &prevsync,
                     int &lastseen_offset, int &rds_bit_cont, int &lastseen_offset_cont, int &block_distance,
                     int &block_number, int &block_bit_cont, int &blocks_cont, int &wrong_blocks_cont,
                     int &group_assembly_started, int &group_good_blocks_cont, const std::vector<int> &decoded_bits);
void start_frame_sync(unsigned int &idx, std::vector<int> &stream, std::vector<int> &sync_state_bits, uint64_t &reg,
                      uint64_t &chars, uint64_t &output, bool &first_time, std::deque<std::string> &window);

#endif
