// rds_text_driver.cpp -- test driver for the host RDS frame layer (real-time-sdr_amd/host/rds_frame.cpp).
// stdin: one line per block, the block's decoded RDS bits as 0/1 characters ("-" for a block that
// does not decode). It accumulates decoded bits and runs start_frame_sync every 15 decoding blocks,
// as the reference's rds stage does (rds.cpp:181-189); parse() prints the text to stderr.
#include <deque>
#include <iostream>
#include <string>
#include <vector>

#include "rds_utilities.h"

int main() {
    uint64_t reg = 0, chars = 0, output = 0;
    bool first_time = true;
    int decoder_cont = 0;
    unsigned int idx = 0;
    std::deque<std::string> window;
    std::vector<int> stream, state;
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line == "-") continue;
        decoder_cont++;
        for (char ch : line) stream.push_back(ch == '1');
        if (decoder_cont == 15) {
            start_frame_sync(idx, stream, state, reg, chars, output, first_time, window);
            decoder_cont = 0;
            idx = 0;
            stream.clear();
        }
    }
    return 0;
}
